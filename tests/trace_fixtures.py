"""Reading the converted reference traces (tests/golden/make_trace_fixtures.py) for the GPU replay
(tests/test_gpu_traces.py) and its CPU-side checks.  Test infrastructure only."""
import collections
import json
import os
import xml.etree.ElementTree as ET

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TR = os.path.join(ROOT, "tests", "golden", "traces")
IDX = json.load(open(os.path.join(TR, "index.json")))


def map_size(map_rel):
    r = ET.parse(os.path.join(ROOT, map_rel)).getroot()
    return int(r.get("height")), int(r.get("width"))


GROUPS = collections.defaultdict(list)
for _e in IDX:
    GROUPS[map_size(_e["map"])].append(_e)
SIZES = sorted(GROUPS)


def parse(text):
    """Fixture text -> [(time, (r0, r1), units int32 [n][6] (type, player, x, y, hp, res), actions)] per
    entry; an action is the issue row (player, x, y, type, parameter, target x, target y, unit type) —
    its unit ID resolved to that unit's player and position in the entry's own snapshot."""
    tok = text.split()
    assert tok[0] == "TRACE"
    n, i, out = int(tok[1]), 2, []
    for _ in range(n):
        assert tok[i] == "E"
        time = int(tok[i + 1])
        r = (int(tok[i + 3]), int(tok[i + 4]))
        nu = int(tok[i + 6])
        i += 7
        units, where = [], {}
        for _ in range(nu):
            t, uid, pl, x, y, res, hp = (int(v) for v in tok[i + 1:i + 8])
            units.append((t, pl, x, y, hp, res))
            where[uid] = (pl, x, y)
            i += 8
        na = int(tok[i + 1])
        i += 2
        acts = []
        for _ in range(na):
            uid, t, prm, ax, ay, ut = (int(v) for v in tok[i + 1:i + 7])
            pl, x, y = where[uid]
            acts.append((pl, x, y, t, prm, ax, ay, ut))
            i += 7
        out.append((time, r, np.array(units, dtype=np.int32).reshape(-1, 6), acts))
    return out


def issue_rows(acts):
    """TestTracesIntegrity.java:101-117: player 0's actions in trace order, then player 1's."""
    return [a for a in acts if a[0] == 0] + [a for a in acts if a[0] == 1]


def check_vs_trace(dump, entry, tag):
    time, (r0, r1), units, _ = entry
    assert dump[0] == time, f"{tag}: time {dump[0]} vs {time}"
    assert (dump[2], dump[3]) == (r0, r1), f"{tag}: player resources {dump[2:4]} vs {(r0, r1)}"
    nu = int(dump[4])
    assert nu == len(units), f"{tag}: unit count {nu} vs {len(units)}"
    got = dump[5:5 + 6 * nu].reshape(-1, 6)
    bad = np.nonzero((got != units).any(axis=1))[0]
    assert len(bad) == 0, f"{tag}: unit {bad[0]} {got[bad[0]].tolist()} vs trace {units[bad[0]].tolist()}"
