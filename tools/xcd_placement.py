#!/usr/bin/env python3
"""Diagnostic: is a game's XCD (HW_REG_XCC_ID of the wave that steps it) the same in consecutive
step launches?  Uses the timing build (libmrts_timing.so: per-game placement words of the last
launch).  Prints, for 6 consecutive launches, the fraction of games whose XCD equals their XCD in
the previous launch, and the (block - xcd) mod 8 offsets seen per launch."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from microrts_amd import _lib  # noqa: E402

L = _lib.load(os.path.join(ROOT, "microrts_amd", "libmrts_timing.so"))
L.mrts_phase_spans.argtypes = [ctypes.c_void_p, ctypes.c_int]
from microrts_amd import DeviceVecEnv  # noqa: E402

E = 4096
SEED = 0x5EEDC0DE
env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, "maps/16x16/basesWorkers16x16.xml")] * (2 * E), seed=SEED)
env.reset()
env.random_policy(SEED, 0)
env.rollout_fused(SEED, 1, 200)
env.synchronize()
prev = None
for k in range(6):
    env.step_fused(SEED, 201 + k)
    env.synchronize()
    sp = (ctypes.c_ulonglong * (3 * E))()
    _lib.check(L.mrts_phase_spans(sp, E))
    place = np.array(sp[2 * E:3 * E], dtype=np.uint64)
    xcc = ((place >> np.uint64(32)) & np.uint64(15)).astype(np.int64)
    offs = np.unique((np.arange(E) - xcc) % 8, return_counts=True)
    out = {"launch": k, "offsets_block_minus_xcd_mod8": dict(zip(offs[0].tolist(), offs[1].tolist()))}
    if prev is not None:
        out["same_xcd_as_previous_launch"] = float((xcc == prev).mean())
    print(json.dumps(out), flush=True)
    prev = xcc
env.close()
