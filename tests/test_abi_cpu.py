"""CPU-side checks of the drop-in boundary: libmrts.so loads and exports every symbol include/mrts.h
declares; the Python mirror validates its arguments (no GPU compute is called here)."""
import ctypes
import os
import re

import pytest

from microrts_amd import _lib
from microrts_amd.vec_client import UnitTypeTable, _check_rfs, _bot_kind

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "mrts.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mrts_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_python_exports():
    assert header_symbols() == sorted(_lib.EXPORTS)


def test_library_loads_and_exports_every_symbol():
    L = _lib.load()
    for name in header_symbols():
        assert hasattr(L, name), name
        assert ctypes.cast(getattr(L, name), ctypes.c_void_p).value


def test_config_struct_layout():
    # mrts_config: 6 int32, pointer, pointer, int32, uint64, int32 (natural alignment)
    assert ctypes.sizeof(_lib.MrtsConfig) == 104
    assert _lib.MrtsConfig.seed.offset == 56
    assert _lib.MrtsConfig.mask_delta.offset == 68
    assert _lib.MrtsConfig.reward_kinds.offset == 72 and _lib.MrtsConfig.n_rewards.offset == 80
    assert _lib.MrtsConfig.forward_model.offset == 84 and _lib.MrtsConfig.utt_json.offset == 88
    assert _lib.MrtsConfig.max_units.offset == 96


def test_config_struct_matches_the_c_header(tmp_path):
    """offsetof / sizeof of every mrts_config member as the C compiler lays out include/mrts.h"""
    import shutil
    import subprocess

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    names = [f[0] for f in _lib.MrtsConfig._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mrts.h"\nint main(void) {\n'
                   + "".join(f'  printf("%zu\\n", offsetof(mrts_config, {n}));\n' for n in names)
                   + '  printf("%zu\\n", sizeof(mrts_config));\n  return 0;\n}\n')
    exe = tmp_path / "layout"
    subprocess.check_call([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [getattr(_lib.MrtsConfig, n).offset for n in names] + [ctypes.sizeof(_lib.MrtsConfig)]
    assert got == want


def test_argument_validation():
    with pytest.raises(NotImplementedError):
        _check_rfs(["ScoreRewardFunction"])
    assert _check_rfs(None) == [0]
    assert _check_rfs(["WinLossRewardFunction", "ResourceGatherRewardFunction", "ProduceWorkerRewardFunction",
                       "ProduceBuildingRewardFunction", "AttackRewardFunction", "ProduceCombatUnitRewardFunction",
                       "CloserToEnemyBaseRewardFunction", "CloserToEnemyUnitRewardFunction"]) == list(range(8))

    class AttackRewardFunction:  # an instance named like the Java class is accepted (JPype proxies)
        pass

    assert _check_rfs([AttackRewardFunction()]) == [4]
    with pytest.raises(NotImplementedError):
        _bot_kind("WorkerRush")
    assert _bot_kind("PassiveAI") == 0
    with pytest.raises(ValueError):
        UnitTypeTable(4)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError):
        _lib.load.__wrapped__(str(tmp_path / "nope.so")) if hasattr(_lib.load, "__wrapped__") else _load_missing(tmp_path)


def _load_missing(tmp_path):
    saved = _lib._lib
    _lib._lib = None
    try:
        _lib.load(str(tmp_path / "nope.so"))
    finally:
        _lib._lib = saved


def test_vecclient_mirror_rejects_missing_bots():
    """Java indexes a_ai2s[i] / a_ai1s[i] / mapPaths[i] for every env (JNIGridnetVecClient.java:119-123,
    163-165): a null or short array throws there, so the mirror raises before creating anything."""
    from microrts_amd import JNIGridnetVecClient

    m = "maps/8x8/basesWorkers8x8.xml"
    with pytest.raises(ValueError, match="a_ai2s"):
        JNIGridnetVecClient(2, 2, 100, None, "", [m] * 4)
    with pytest.raises(ValueError, match="a_ai2s"):
        JNIGridnetVecClient(2, 2, 100, None, "", [m] * 4, ["PassiveAI"])
    with pytest.raises(ValueError, match="a_ai1s"):
        JNIGridnetVecClient.bots(100, None, "", [m] * 2, ["PassiveAI"], ["PassiveAI"] * 2)
    with pytest.raises(ValueError, match="map paths"):
        JNIGridnetVecClient(4, 0, 100, None, "", [m] * 2)  # Java reads mapPaths[2]
    with pytest.raises(ValueError, match="map paths"):
        JNIGridnetVecClient(2, 2, 100, None, "", [m] * 3, ["PassiveAI"] * 2)  # mapPaths[3]


def test_vecclient_mirror_map_index_is_javas():
    """the mirror requires exactly the mapPaths indices Java reads — [i*2] per self-play
    client (JNIGridnetVecClient.java:119), [a_num_selfplayenvs + i] per bot env (:123), [0] for the
    storage sizing (:127) — so a self-play-only client with n-1 paths is accepted like Java's."""
    from microrts_amd.vec_client import _last_map_index

    assert _last_map_index(4, 0) == 2  # 3 paths suffice for 4 self-play slots
    assert _last_map_index(2, 0) == 0
    assert _last_map_index(0, 3) == 2
    assert _last_map_index(2, 2) == 3
    assert _last_map_index(0, 0) == 0


def _utt_with(sight_of_worker):
    import json

    t = json.load(open(os.path.join(ROOT, "tests", "golden", "utts", "TestUnitTypeTable.json")))
    for ut in t["unitTypes"]:
        if ut["name"] == "Worker":
            ut["sightRadius"] = sight_of_worker
    return json.dumps(t)


def test_po_random_biased_needs_sight_covering_actions():
    """the GPU RandomBiasedAI computes an owned unit's actions on the full cell map, which
    equals its PartiallyObservableGameState view (JNIGridnetClient.java:164-173) only if the unit sees
    every cell it can act on.  A table with a blind Worker is refused at create (before any GPU
    call); the same table without PO, or with PassiveAI, passes this check."""
    from microrts_amd.vec_client import _Handle

    m = "maps/8x8/basesWorkers8x8.xml"
    blind = UnitTypeTable.fromJSON(_utt_with(0))
    with pytest.raises(RuntimeError, match="sightRadius"):
        _Handle(0, 2, 100, [m] * 2, ["RandomBiasedAI"] * 2, blind, True, 0, 0, 0)
    # the check is specific: no error of that kind for PassiveAI or full observability (these
    # then fail only on the missing GPU, or succeed on a GPU box)
    for ai, po in (("PassiveAI", True), ("RandomBiasedAI", False)):
        try:
            h = _Handle(0, 2, 100, [m] * 2, [ai] * 2, blind, po, 0, 0, 0)
            h.close()
        except RuntimeError as e:
            assert "sightRadius" not in str(e)
    ok = UnitTypeTable.fromJSON(_utt_with(1))
    try:
        _Handle(0, 2, 100, [m] * 2, ["RandomBiasedAI"] * 2, ok, True, 0, 0, 0).close()
    except RuntimeError as e:
        assert "sightRadius" not in str(e)
