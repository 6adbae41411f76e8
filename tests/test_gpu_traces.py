"""The reference's own recorded games replayed through the HIP kernels.

data/traces/**/trace_0.zip holds 280 games (LightRush / PortfolioAI on all 140 maps, UTT
VERSION_ORIGINAL), converted as data by tests/golden/make_trace_fixtures.py.  The reference replays
them with test/microrts/TestTracesIntegrity.java:72-127: cycle() up to each entry's time, then
issueSafe(player 0's actions), issueSafe(player 1's actions), where every action binds to the first
live unit at its unit's (x, y) (rts/GameState.java:356-382).  Here that loop runs on the product
kernels: mrts_trace_step (k_env MODE_TRACE) issues an entry's actions through the kernels' own
legality / issueSafe / issue code and cycles the game to the next entry's time.  At every one of the
17,085 entries:

* the GPU state must equal the trace's recorded PhysicalGameState (time, players' resources, every
  unit in list order: type, player, x, y, hit points, carried resources) — a pin on reference-held
  vectors, stricter than the reference's own test, which checks only issueSafe's return value;
* the canonical dump (including the pending assignments in LinkedHashMap order, which the trace does
  not record) must equal the CPU oracle's replay of the same trace;
* issueSafe's return value must equal the trace's "contains real actions" (the reference's assertion)
  and the oracle's, and no cycle may follow one that ended the game (the reference's assertFalse).

Every map size runs on the generic kernel; the 8x8 and 16x16 traces also run on the specialised
instances the benchmark shapes use (compile-time map dimensions).
"""
import gzip
import os

import numpy as np
import pytest

from tests import oracle_py

pytestmark = pytest.mark.gpu

from tests.trace_fixtures import GROUPS, IDX, ROOT, SIZES, TR, check_vs_trace, map_size, parse, issue_rows

TRACE_ISSUED, TRACE_GAMEOVER, TRACE_NO_UNIT = 1, 2, 4


def _replay(entries_list, maps, generic, oracle=None, corrupt=None):
    """Replay the traces of one map size as the games of one forward-model handle.  Returns the number
    of entries checked; with `corrupt`, returns at the first mismatch instead (index of that entry)."""
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from microrts_amd import ForwardModel

    n = len(entries_list)
    H, W = map_size(maps[0])
    mu = 1024 if H * W > 64 * 64 else 0
    fm = ForwardModel(n, [os.path.join(ROOT, m) for m in maps], policies=("PassiveAI", "PassiveAI"), max_units=mu)
    checked = 0
    try:
        for k in range(max(len(e) for e in entries_list) + 1):
            rows = [issue_rows(e[k - 1][3]) if 0 < k <= len(e) else [] for e in entries_list]
            until = [e[k][0] if k < len(e) else 0 for e in entries_list]
            npair = max(1, max(len(r) for r in rows))
            pairs = np.full((n, npair, 8), -1, dtype=np.int32)
            for g, r in enumerate(rows):
                if r:
                    pairs[g, :len(r)] = np.array(r, dtype=np.int32)
            flags = fm.trace_step(pairs, until, generic=generic)
            for g, e in enumerate(entries_list):
                try:
                    checked += _check_entry(fm, g, e, k, int(flags[g]), oracle[g] if oracle else None, f"{maps[g]} entry {k}")
                except AssertionError:
                    if corrupt:
                        return k
                    raise
        assert not fm.error_flags().any()
    finally:
        fm.close()
    return None if corrupt else checked


def _check_entry(fm, g, e, k, flags, oracle, tag):
    assert not flags & TRACE_NO_UNIT, f"{tag}: an action names a cell without a unit"
    assert not flags & TRACE_GAMEOVER, f"{tag}: cycle after gameover"
    if 0 < k <= len(e):  # TestTracesIntegrity.java:124 — and the oracle's replay agrees
        if e[k - 1][3]:
            real = any(a[3] != 0 for a in e[k - 1][3])
            assert bool(flags & TRACE_ISSUED) == real, f"{tag}: issueSafe returned {not real}"
        if oracle is not None:
            assert bool(flags & TRACE_ISSUED) == bool(oracle[1][k - 1]), f"{tag}: issued vs oracle"
    if k >= len(e):
        return 0
    d = fm.dump_state(g)
    check_vs_trace(d, e[k], tag)
    if oracle is not None:
        assert np.array_equal(d, oracle[0][k]), f"{tag}: state (with assignments) differs from the oracle's replay"
    return 1


def _load(group):
    texts = [gzip.open(os.path.join(TR, e["fixture"]), "rt").read() for e in group]
    entries = [parse(t) for t in texts]
    for e, g in zip(entries, group):
        assert len(e) == g["entries"]
    oracle = [oracle_py.trace_dumps(os.path.join(ROOT, g["map"]), t) for g, t in zip(group, texts)]
    return entries, oracle


CASES = [(s, True) for s in SIZES] + [(s, False) for s in SIZES if s in ((8, 8), (16, 16))]


@pytest.mark.parametrize("size,generic", CASES, ids=[f"{h}x{w}-{'generic' if g else 'specialised'}" for (h, w), g in CASES])
def test_reference_traces_on_gpu(size, generic):
    group = GROUPS[size]
    entries, oracle = _load(group)
    n = _replay(entries, [g["map"] for g in group], generic, oracle)
    assert n == sum(g["entries"] for g in group)


def test_all_reference_traces_covered():
    """The cases above cover every fixture: 280 traces, 17,085 entries, 140 maps."""
    assert sum(len(GROUPS[s]) for s in SIZES) == len(IDX) == 280
    assert sum(e["entries"] for e in IDX) == 17085
    assert len({e["map"] for e in IDX}) == 140


def test_trace_replay_detects_a_wrong_action():
    """The comparison is not vacuous: the first MOVE of a 16x16 trace turned into the opposite direction
    (a legal move onto the cell the unit left, or NONE) makes a later entry differ from the trace."""
    group = [e for e in GROUPS[(16, 16)] if "basesWorkers16x16" in e["map"]][:1]
    entries, _ = _load(group)
    e = entries[0]
    for k, ent in enumerate(e):
        mv = [i for i, a in enumerate(ent[3]) if a[3] == 1]
        if mv:
            a = list(ent[3][mv[0]])
            a[4] = (a[4] + 2) % 4
            ent[3][mv[0]] = tuple(a)
            break
    bad = _replay(entries, [group[0]["map"]], True, corrupt=True)
    assert bad is not None and bad > k, "the corrupted action went unnoticed"
