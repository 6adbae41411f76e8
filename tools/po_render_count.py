#!/usr/bin/env python3
"""Diagnostic (libmrts_ablate.so): (view, chunk) items the partially observable renderer writes per
game-step, and how many renders ran as deltas — one launch per step vs multi-step launches, c5."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from microrts_amd import _lib  # noqa: E402

L = _lib.load(os.path.join(ROOT, "microrts_amd", "libmrts_ablate.so"))
L.mrts_get_dbg.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.mrts_set_ablate.argtypes = [ctypes.c_uint]
L.mrts_set_ablate(1 << 24)  # AB_COUNT: the render-item counters (contended atomics: diagnostics only)
from microrts_amd import DeviceVecEnv  # noqa: E402

SEED = 0x5EEDC0DE
E = int(os.environ.get("E", 256))
env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, "maps/BWDistantResources32x32.xml")] * (2 * E), seed=SEED,
                   partial_obs=True, max_units=256)
env.reset()
env.random_policy(SEED, 0)
env.rollout_fused(SEED, 1, 300)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 4)()
for multi in (False, True, False, True):
    env.set_multi_step(multi)
    env.rollout_fused(SEED, 301, 3)
    torch.cuda.synchronize()
    L.mrts_get_dbg(buf, 1)
    env.rollout_fused(SEED, 304, 50)
    torch.cuda.synchronize()
    L.mrts_get_dbg(buf, 1)
    print(json.dumps({"multi": multi, "renders": buf[1], "delta_renders": buf[2],
                      "items_per_render": round(buf[0] / max(1, buf[1]), 1)}), flush=True)
