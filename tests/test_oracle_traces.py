"""Pin the CPU oracle against the reference's own golden vectors.

* every data/traces/**/trace_0.zip of the reference (280 LightRush / PortfolioAI games,
  converted by tests/golden/make_trace_fixtures.py) is replayed with the rule of
  test/microrts/TestTracesIntegrity.java:72-127, and — stricter than the reference's
  test — the full PhysicalGameState (players' resources; units in list order: type,
  player, x, y, hp, carried resources) must equal the trace's snapshot at every entry;
* every map under maps/ loads (test/microrts/TestLoadingMaps.java:24-51).
"""
import ctypes
import glob
import gzip
import json
import os

import pytest

from tests import oracle_py

ROOT = oracle_py.ROOT
IDX = json.load(open(os.path.join(ROOT, "tests", "golden", "traces", "index.json")))


@pytest.mark.parametrize("entry", IDX, ids=[e["fixture"] for e in IDX])
def test_trace_strict_replay(oracle_lib, entry):
    txt = gzip.open(os.path.join(ROOT, "tests", "golden", "traces", entry["fixture"]), "rt").read()
    msg = ctypes.create_string_buffer(1024)
    n = oracle_lib.oref_trace_replay(os.path.join(ROOT, entry["map"]).encode(), txt.encode(), msg, 1024)
    assert n == entry["entries"], msg.value.decode()


def test_trace_replay_detects_corruption(oracle_lib):
    """A one-unit hp change in a snapshot must be reported (the check is not vacuous)."""
    e = IDX[100]
    lines = gzip.open(os.path.join(ROOT, "tests", "golden", "traces", e["fixture"]), "rt").read().split("\n")
    ulines = [i for i, l in enumerate(lines) if l.startswith("U ")]
    i = ulines[len(ulines) // 2]
    parts = lines[i].split()
    parts[7] = str(int(parts[7]) + 1)
    lines[i] = " ".join(parts)
    msg = ctypes.create_string_buffer(1024)
    n = oracle_lib.oref_trace_replay(os.path.join(ROOT, e["map"]).encode(), "\n".join(lines).encode(), msg, 1024)
    assert n == -1 and b"hp" in msg.value


def test_trace_dumps_follow_the_fixtures(oracle_lib):
    """The per-entry oracle dumps the GPU replay compares against (oref_trace_dumps) hold the traces'
    own snapshots, and issueSafe's return value equals "contains real actions" at every entry with
    actions (TestTracesIntegrity.java:124) — which also checks tests/trace_fixtures.parse."""
    from tests import trace_fixtures as T

    n = 0
    for e in IDX:
        text = gzip.open(os.path.join(ROOT, "tests", "golden", "traces", e["fixture"]), "rt").read()
        ents = T.parse(text)
        dumps, issued = oracle_py.trace_dumps(os.path.join(ROOT, e["map"]), text)
        assert len(ents) == len(dumps) == e["entries"]
        for k, (ent, d) in enumerate(zip(ents, dumps)):
            T.check_vs_trace(d, ent, f"{e['fixture']} entry {k}")
            if ent[3]:
                assert bool(issued[k]) == any(a[3] != 0 for a in ent[3])
            n += 1
    assert n == 17085


MAPS = sorted(glob.glob(os.path.join(ROOT, "maps", "**", "*.xml"), recursive=True))


def test_all_maps_load(oracle_lib):
    assert len(MAPS) == 140
    for m in MAPS:
        rel = os.path.relpath(m, ROOT)
        v = oracle_py.OracleVecClient(2, 0, 100, [rel, rel])
        obs, _, _ = v.reset()
        assert obs.shape[2:] == (v.H, v.W)
        v.close()
