#!/usr/bin/env python3
"""Diagnostic: how unevenly the SIMDs finish a multi-step launch (libmrts_span.so, built with
`make -C microrts_amd/csrc span`; never loaded by the package).  Runs the c3 workload's burn-in, then
one K-step multi-step rollout, and reports per-game start / end (s_memrealtime, 100 MHz) with each
wave's placement (HW_ID / XCC_ID): the spread of the games' end times and of the per-SIMD last end —
what perfectly balanced SIMDs would save over the slowest one."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from microrts_amd import _lib  # noqa: E402

L = _lib.load(os.path.join(ROOT, "microrts_amd", "libmrts_span.so"))
L.mrts_phase_spans.argtypes = [ctypes.c_void_p, ctypes.c_int]
from microrts_amd import DeviceVecEnv  # noqa: E402

E = int(os.environ.get("E", 4096))
K = int(os.environ.get("K", 200))
SEED = 0x5EEDC0DE
MAP = os.environ.get("MAP", "maps/16x16/basesWorkers16x16.xml")
PO = os.environ.get("PO", "0") == "1"
env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, MAP)] * (2 * E), seed=SEED, partial_obs=PO,
                   max_units=int(os.environ.get("MAXU", 0)))
env.reset()
env.random_policy(SEED, 0)
env.rollout_fused(SEED, 1, 1000)
torch.cuda.synchronize()
for rep in range(3):
    first = 1001 + rep * K
    env.rollout_fused(SEED, first, K)
    torch.cuda.synchronize()
    sp = (ctypes.c_ulonglong * (11 * E))()  # mrts_phase_spans writes [11][E]
    _lib.check(L.mrts_phase_spans(sp, E))
    st = np.array(sp[0:E], dtype=np.float64)
    en = np.array(sp[E:2 * E], dtype=np.float64)
    place = np.array(sp[2 * E:3 * E], dtype=np.uint64)
    hw = (place & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcc = ((place >> np.uint64(32)) & np.uint64(15)).astype(np.int64)
    nu_end = ((place >> np.uint64(48)) & np.uint64(255)).astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    t0 = st.min()
    end = (en - t0) / 100.0  # us
    dur = (en - st) / 100.0
    uniq, inv = np.unique(key, return_inverse=True)
    simd_last = np.zeros(len(uniq))
    np.maximum.at(simd_last, inv, end)
    simd_units = np.bincount(inv, weights=nu_end)
    if os.environ.get("DUMP"):  # raw per-game arrays for offline analysis
        np.savez(f"{os.environ['DUMP']}_E{E}_K{K}_rep{rep}.npz", end=end, dur=dur, nu_end=nu_end, key=key)
    print(json.dumps({"K": K, "rep": rep, "launch_us": round(float(end.max()), 1),
                      "per_step_us": round(float(end.max()) / K, 3),
                      "game_end_us": {"min": round(float(end.min()), 1), "mean": round(float(end.mean()), 1),
                                      "p99": round(float(np.percentile(end, 99)), 1), "max": round(float(end.max()), 1)},
                      "start_spread_us": round(float((st.max() - t0) / 100.0), 2),
                      "simds": int(len(uniq)), "games_per_simd": np.bincount(np.bincount(inv)).tolist(),
                      "simd_last_end_us": {"mean": round(float(simd_last.mean()), 1), "p50": round(float(np.median(simd_last)), 1),
                                           "p99": round(float(np.percentile(simd_last, 99)), 1), "max": round(float(simd_last.max()), 1)},
                      "corr_simd_units_end": round(float(np.corrcoef(simd_units, simd_last)[0, 1]), 3),
                      "corr_game_units_dur": round(float(np.corrcoef(nu_end, dur)[0, 1]), 3)}), flush=True)
