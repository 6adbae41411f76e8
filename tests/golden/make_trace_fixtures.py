#!/usr/bin/env python3
"""Convert the reference's golden game traces into compact oracle fixtures.

Input : /root/reference/data/traces/<map>/<AI>/trace_0.zip  (280 zipped XML traces,
        written by src/tests/GenerateTestTraces.java:40-140 and replayed by
        test/microrts/TestTracesIntegrity.java:72-127).  They are DATA files held by
        the reference's own test; they are parsed here as data (xml.etree, no code).
Output: tests/golden/traces/<map path with '/' -> '__'>__<AI>.trace.gz  and  index.json

Fixture text format (whitespace separated, consumed by oracle_capi.cpp:oref_trace_replay):
    TRACE <n_entries>
    per entry:
      E <time>
      P <resources p0> <resources p1>
      N <n_units>
      U <typeID> <unitID> <player> <x> <y> <resources> <hitpoints>      (n_units lines, list order)
      A <n_actions>
      a <unitID> <type> <parameter> <x> <y> <unitTypeID or -1>         (n_actions lines, trace order)
Defaults follow rts/UnitAction.java:590-610 (parameter -1, x 0, y 0, unitType null).

Run once in the build container (the reference is not on the GPU box):
    python tests/golden/make_trace_fixtures.py
"""
import gzip
import json
import os
import sys
import xml.etree.ElementTree as ET
import zipfile

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "traces")
TYPES = ["Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"]
# VERSION_ORIGINAL constants (rts/units/UnitTypeTable.java:104-289) — every trace must embed these
V1 = {
    "Resource": dict(cost=1, hp=1, produceTime=10, moveTime=10, attackTime=10, harvestTime=10),
    "Base": dict(cost=10, hp=10, produceTime=250),
    "Barracks": dict(cost=5, hp=4, produceTime=200),
    "Worker": dict(cost=1, hp=1, produceTime=50, moveTime=10, attackTime=5, harvestTime=20, minDamage=1, maxDamage=1),
    "Light": dict(cost=2, hp=4, produceTime=80, moveTime=8, attackTime=5, minDamage=2, maxDamage=2),
    "Heavy": dict(cost=2, hp=4, produceTime=120, moveTime=12, attackTime=5, minDamage=4, maxDamage=4),
    "Ranged": dict(cost=2, hp=1, produceTime=100, moveTime=10, attackTime=5, minDamage=1, maxDamage=1, attackRange=3),
}


def convert(zpath):
    with zipfile.ZipFile(zpath) as z:
        xml = z.read(z.namelist()[0])
    root = ET.fromstring(xml)
    utt = root.find("rts.units.UnitTypeTable")
    assert utt.get("moveConflictResolutionStrategy") == "1"
    for ut in utt.findall("rts.units.UnitType"):
        name = ut.get("name")
        assert TYPES.index(name) == int(ut.get("ID"))
        for k, v in V1[name].items():
            assert int(ut.get(k)) == v, (zpath, name, k)
    lines = []
    entries = root.find("entries").findall("rts.TraceEntry")
    lines.append("TRACE %d" % len(entries))
    for e in entries:
        pgs = e.find("rts.PhysicalGameState")
        players = pgs.find("players").findall("rts.Player")
        assert [int(p.get("ID")) for p in players] == [0, 1]
        lines.append("E %d" % int(e.get("time")))
        lines.append("P %d %d" % tuple(int(p.get("resources")) for p in players))
        units = pgs.find("units").findall("rts.units.Unit")
        lines.append("N %d" % len(units))
        for u in units:
            lines.append("U %d %s %s %s %s %s %s" % (TYPES.index(u.get("type")), u.get("ID"), u.get("player"), u.get("x"),
                                                   u.get("y"), u.get("resources"), u.get("hitpoints")))
        acts = e.find("actions").findall("action")
        lines.append("A %d" % len(acts))
        for a in acts:
            ua = a.find("UnitAction")
            ut = ua.get("unitType")
            lines.append("a %s %s %s %s %s %d" % (a.get("unitID"), ua.get("type"), ua.get("parameter", "-1"), ua.get("x", "0"),
                                                 ua.get("y", "0"), TYPES.index(ut) if ut else -1))
    return "\n".join(lines) + "\n", len(entries)


def main():
    os.makedirs(OUT, exist_ok=True)
    index = []
    root = os.path.join(REF, "data", "traces")
    for dirpath, _, files in sorted(os.walk(root)):
        for f in sorted(files):
            if not f.endswith(".zip"):
                continue
            zpath = os.path.join(dirpath, f)
            rel = os.path.relpath(zpath, root)  # <map...>/<AI>/trace_0.zip
            parts = rel.split(os.sep)
            ai, mapparts = parts[-2], parts[:-2]
            mapfile = "maps/" + "/".join(mapparts) + ".xml"
            if not os.path.exists(os.path.join(REF, mapfile)):
                print("skip (no map):", rel)
                continue
            text, n = convert(zpath)
            name = "__".join(mapparts) + "__" + ai.split("_")[0] + ".trace.gz"
            with gzip.open(os.path.join(OUT, name), "wt", compresslevel=9) as g:
                g.write(text)
            index.append(dict(fixture=name, map=mapfile, ai=ai, entries=n, source="data/traces/" + rel.replace(os.sep, "/")))
    with open(os.path.join(OUT, "index.json"), "w") as fp:
        json.dump(index, fp, indent=1)
    print("wrote", len(index), "fixtures")


if __name__ == "__main__":
    sys.exit(main())
