#!/usr/bin/env python3
"""Diagnostic: where a single-step c3 launch (one k_env launch per step, the neural-learner
form) spends its ~19 us, from the span build (libmrts_span.so, `make -C microrts_amd/csrc span`; never loaded
by the package): per game the wave's start and end and 8 milestones (s_memrealtime, 100 MHz, lane 0 of the
wave): 20 = state load issued, 21 = state in LDS, 1 = rows decoded, 3 = both players issued, 4 = cycle done,
5 = outcome / reward / reset done, 6 = observation written, 9 = masks + policy rows written; then the store.
Prints per launch: the launch span, the start spread, the mean time of each phase, the games' end spread and
the per-SIMD last end; and the same for one K = 20 multi-step launch (per step).  One JSON line per launch."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from microrts_amd import _lib  # noqa: E402

STEPM = os.environ.get("MILES") == "step"  # libmrts_span_step.so: iteration start / rows unpacked instead of the load
L = _lib.load(os.path.join(ROOT, "microrts_amd", "libmrts_span_step.so" if STEPM else "libmrts_span.so"))
L.mrts_phase_spans.argtypes = [ctypes.c_void_p, ctypes.c_int]
from microrts_amd import DeviceVecEnv  # noqa: E402

CFG = os.environ.get("CFG", "c3")  # c5: 2048 partially observable 32x32 games (render helper wave)
E = int(os.environ.get("E", 4096 if CFG == "c3" else 2048))
SEED = 0x5EEDC0DE
MAP = os.path.join(ROOT, "maps/16x16/basesWorkers16x16.xml" if CFG == "c3" else "maps/BWDistantResources32x32.xml")
MILES = (["it_start", "rows_index", "decoded", "issued", "cycled", "outcome", "obs", "masks"] if STEPM else
         ["load_issued", "load_done", "decoded", "issued", "cycled", "outcome", "obs", "masks"])


def spans():
    sp = (ctypes.c_ulonglong * (11 * E))()
    _lib.check(L.mrts_phase_spans(sp, E))
    a = np.array(sp, dtype=np.float64).reshape(11, E)
    return a[0], a[1], a[2].astype(np.uint64), a[3:]


def main():
    po = CFG == "c5"
    env = DeviceVecEnv(2 * E, 0, 2000, [MAP] * (2 * E), seed=SEED, partial_obs=po, max_units=256 if po else 0)
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, 1000)
    torch.cuda.synchronize()
    k = 1001
    for mode, K in (("single", 1), ("single", 1), ("single", 1), ("multi", 20)):
        env.set_multi_step(mode == "multi")
        env.rollout_fused(SEED, k, K)
        k += K
        torch.cuda.synchronize()
        st, en, place, mi = spans()
        t0 = st.min()
        us = lambda v: (v - t0) / 100.0  # noqa: E731
        hw = (place & np.uint64(0xFFFFFFFF)).astype(np.int64)
        xcc = ((place >> np.uint64(32)) & np.uint64(15)).astype(np.int64)
        key = ((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 64 + ((hw >> 8) & 15) * 4 + ((hw >> 4) & 3)
        uniq, inv = np.unique(key, return_inverse=True)
        last = np.zeros(len(uniq))
        np.maximum.at(last, inv, us(en))
        out = {"mode": mode, "K": K, "launch_us": round(float(us(en).max()), 2),
               "start_spread_us": round(float(us(st).max()), 2), "game_us_mean": round(float(((en - st) / 100).mean()), 2),
               "game_end_us": {"mean": round(float(us(en).mean()), 2), "max": round(float(us(en).max()), 2)},
               "simd_last_end_us": {"mean": round(float(last.mean()), 2), "max": round(float(last.max()), 2)}}
        if mode == "multi" and os.environ.get("PLACEMENT"):  # which blocks share a SIMD (game waves only)
            groups = [np.flatnonzero(inv == u) for u in range(len(uniq))]
            sizes = np.bincount([len(gq) for gq in groups])
            offs = {}
            for gq in groups:
                t = tuple(int(x) for x in (gq - gq[0]))
                offs[t] = offs.get(t, 0) + 1
            top = sorted(offs.items(), key=lambda kv: -kv[1])[:4]
            xcc_of = (uniq // (8 * 2 * 64)).astype(np.int64)  # key = ((xcc * 8 + se) * 2 + sh) * 64 + cu * 4 + simd
            out["per_xcd"] = [{"xcd": int(x), "game_end_mean_us": round(float(us(en)[xcc == x].mean()), 2),
                               "simd_last_end_mean_us": round(float(last[xcc_of == x].mean()), 2),
                               "simd_last_end_max_us": round(float(last[xcc_of == x].max()), 2)} for x in np.unique(xcc)]
            out["placement"] = {"simds": len(uniq), "games_per_simd_hist": sizes.tolist(),
                                "block_offset_patterns": [[list(k), v] for k, v in top],
                                "first_groups": [gq.tolist() for gq in groups[:4]]}
        if mode == "multi":  # the LAST iteration's milestones (each stamp is overwritten per iteration)
            m = {name: v for name, v in zip(MILES, mi)}
            seq = (["it_start", "rows_index"] if STEPM else []) + ["decoded", "issued", "cycled", "outcome", "obs", "masks"]
            ok = np.all([m[n] > 0 for n in seq], axis=0)
            out["last_step_phase_us_mean"] = {b: round(float(((m[b] - m[a]) / 100)[ok].mean()), 3) for a, b in zip(seq, seq[1:])}
            out["last_step_masks_to_end_us"] = round(float(((en - m["masks"]) / 100)[ok].mean()), 3)
        if mode == "single":  # milestones of the (only) step: mean time from the previous milestone
            prev = st
            ph = {}
            for name, m in zip(MILES, mi):
                ok = m > 0
                ph[name] = round(float(((m - prev) / 100)[ok].mean()), 3)
                prev = np.where(ok, m, prev)
            ph["store_to_end"] = round(float(((en - prev) / 100).mean()), 3)
            out["phase_us_mean"] = ph
        print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
