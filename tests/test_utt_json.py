"""JSON unit-type tables (UnitTypeTable.fromJSON :414-433 / toJSON :372-383).

CPU checks: the native tables of versions 1/2/3 written as Java's toJSON and read back; the
reference's own fixture utts/TestUnitTypeTable.json (tests/golden/utts/, data) read with
UnitType.updateFromJSON's quirks; invalid tables rejected; the CPU oracle runs with the same JSON.
GPU parity with JSON tables: tests/test_gpu_parity.py (test_utt_from_json_*)."""
import json
import os

import numpy as np
import pytest

from microrts_amd.vec_client import UnitTypeTable
from tests import oracle_py

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "utts", "TestUnitTypeTable.json")

# rts/units/UnitTypeTable.java:104-289: (cost, hp, minDamage, maxDamage, attackRange, produceTime,
# moveTime, attackTime, harvestTime, sightRadius) per version
V = {
    1: {"Base": (10, 10, 1, 1, 1, 250, 10, 10, 10, 5), "Barracks": (5, 4, 1, 1, 1, 200, 10, 10, 10, 3),
        "Worker": (1, 1, 1, 1, 1, 50, 10, 5, 20, 3), "Light": (2, 4, 2, 2, 1, 80, 8, 5, 10, 2),
        "Heavy": (2, 4, 4, 4, 1, 120, 12, 5, 10, 2), "Ranged": (2, 1, 1, 1, 3, 100, 10, 5, 10, 3)},
    2: {"Base": (10, 10, 1, 1, 1, 200, 10, 10, 10, 5), "Barracks": (5, 4, 1, 1, 1, 100, 10, 10, 10, 3),
        "Worker": (1, 1, 1, 1, 1, 50, 10, 5, 20, 3), "Light": (2, 4, 2, 2, 1, 80, 8, 5, 10, 2),
        "Heavy": (3, 8, 4, 4, 1, 120, 10, 5, 10, 2), "Ranged": (2, 1, 1, 1, 3, 100, 10, 5, 10, 3)},
    # version 3: Base.produceTime has no VERSION_NON_DETERMINISTIC case, so it keeps the default 10
    3: {"Base": (10, 10, 1, 1, 1, 10, 10, 10, 10, 5), "Barracks": (5, 4, 1, 1, 1, 100, 10, 10, 10, 3),
        "Worker": (1, 1, 0, 2, 1, 50, 10, 5, 20, 3), "Light": (2, 4, 1, 3, 1, 80, 8, 5, 10, 2),
        "Heavy": (3, 8, 0, 6, 1, 120, 10, 5, 10, 2), "Ranged": (2, 1, 1, 2, 3, 100, 10, 5, 10, 3)},
}
FIELDS = ("cost", "hp", "minDamage", "maxDamage", "attackRange", "produceTime", "moveTime", "attackTime", "harvestTime",
          "sightRadius")


@pytest.mark.parametrize("version", [1, 2, 3])
def test_builtin_tables_to_json(version):
    t = json.loads(UnitTypeTable(version, 2).toJSON())
    assert t["moveConflictResolutionStrategy"] == 2
    names = [u["name"] for u in t["unitTypes"]]
    assert names == ["Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"]
    for u in t["unitTypes"][1:]:
        assert tuple(u[f] for f in FIELDS) == V[version][u["name"]], u["name"]
        assert u["returnTime"] == 10 and u["harvestAmount"] == 1
    by = {u["name"]: (u["produces"], u["producedBy"]) for u in t["unitTypes"]}
    assert by["Base"] == (["Worker"], ["Worker"]) and by["Worker"] == (["Base", "Barracks"], ["Base"])
    assert by["Barracks"] == (["Light", "Heavy", "Ranged"], ["Worker"]) and by["Light"] == ([], ["Barracks"])


def test_to_json_is_javas_text():
    j = UnitTypeTable().toJSON()  # UnitTypeTable.toJSON / UnitType.toJSON separators, byte for byte
    assert j.startswith('{"moveConflictResolutionStrategy":1,"unitTypes":[{"ID":0, "name":"Resource", "cost":1, "hp":1, ')
    assert '"canAttack":false, "produces":[], "producedBy":[]}, {"ID":1, "name":"Base"' in j
    assert '"produces":["Light", "Heavy", "Ranged"], "producedBy":["Worker"]}' in j
    assert j.endswith("]}]}")


def test_reference_fixture_with_update_quirks():
    text = open(FIXTURE).read()
    src = json.loads(text)
    got = json.loads(UnitTypeTable.fromJSON(text).toJSON())
    for a, b in zip(src["unitTypes"], got["unitTypes"]):
        for k, v in a.items():
            if k == "harvestTime":  # UnitType.updateFromJSON reads harvestTime from "produceTime" (:227)
                assert b[k] == a["produceTime"]
            else:
                assert b[k] == v, (a["name"], k)


def test_round_trip_is_stable_after_one_read():
    once = UnitTypeTable.fromJSON(UnitTypeTable(3, 3).toJSON()).toJSON()
    assert UnitTypeTable.fromJSON(once).toJSON() == once
    assert json.loads(once)["unitTypes"][3]["harvestTime"] == 50  # Worker: produceTime, sic


def test_absent_members_take_update_defaults():
    j = json.dumps({"unitTypes": [{"ID": 0, "name": "Resource", "isResource": True, "produces": [], "producedBy": []},
                                  {"ID": 1, "name": "Worker", "produces": [], "producedBy": []}]})
    w = json.loads(UnitTypeTable.fromJSON(j).toJSON())
    assert w["moveConflictResolutionStrategy"] == 1
    u = w["unitTypes"][1]
    assert (u["harvestAmount"], u["sightRadius"], u["canMove"], u["canAttack"], u["produceTime"]) == (10, 10, False, False, 10)


@pytest.mark.parametrize("bad", [
    "{not json",
    '{"unitTypes": []}',
    '{"unitTypes": [{"ID": 1, "name": "A", "produces": [], "producedBy": []}]}',          # ID != position
    '{"unitTypes": [{"ID": 0, "name": "A", "produces": ["B"], "producedBy": []}]}',       # unknown name
    '{"unitTypes": [{"ID": 0, "name": "A", "attackRange": 4, "produces": [], "producedBy": []}]}',  # K > 80
    '{"moveConflictResolutionStrategy": 4, "unitTypes": [{"ID": 0, "name": "A", "produces": [], "producedBy": []}]}',
    json.dumps({"unitTypes": [{"ID": i, "name": f"T{i}", "produces": [], "producedBy": []} for i in range(9)]}),
])
def test_invalid_tables_rejected(bad):
    with pytest.raises(ValueError):
        UnitTypeTable.fromJSON(bad)


def test_oracle_runs_the_fixture_table():
    text = open(FIXTURE).read()
    ref = oracle_py.OracleVecClient(2, 0, 2000, ["maps/8x8/basesWorkers8x8.xml"] * 2, utt_json=text)
    obs, _, _ = ref.reset()
    base_hp = obs[0, 0][obs[0, 3] == 2]  # plane 3 = type + 1: Base
    assert len(base_hp) == 2 and (base_hp == 10).all()  # the map file's hitpoints, not the table's 50
    for step in range(50):
        m = ref.get_masks(0)
        ref.step(np.stack([oracle_py.policy(m[s], 1, s, step, 0) for s in range(2)]))
    assert ref.env_steps(0) == 50
    ref.close()
