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
