"""Diagnostic: where a k_env<MODE_STEP> game step spends its time (16x16, 4096 games).

Loads the timing build (make -C microrts_amd/csrc timing -> libmrts_timing.so) whose k_env adds
s_memtime stamps between phases; prints mean shader-clock cycles per game step per phase."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from microrts_amd import _lib  # noqa: E402

L = _lib.load(os.path.join(ROOT, "microrts_amd", "libmrts_span.so" if os.environ.get("LIB") == "span" else "libmrts_timing.so"))
L.mrts_phase_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.mrts_phase_spans.argtypes = [ctypes.c_void_p, ctypes.c_int]
from microrts_amd import DeviceVecEnv  # noqa: E402

NAMES = ["load", "predecode", "decode(chain)", "issue", "cycle", "outcome+reset", "obs", "compact", "stashMasks",
         "writeMasks(flush)", "store", "slowIssueBatches(x1000)", "decode(unitLoads)", "decode(baseRes)", "decode(cellRank)",
         "buildIndexCalls(x1000)"] + [f"p{i}" for i in range(16, 32)]
NPH = 32
E = int(os.environ.get("E", 4096))
MAP = os.environ.get("MAP", "maps/16x16/basesWorkers16x16.xml")
PO = os.environ.get("PO", "0") == "1"
SEED = 0x5EEDC0DE


def tail_report(st, en, place):
    """Where the last launch's slow games were: duration vs unit count, and per-SIMD / per-CU load
    (HW_ID: wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13; XCC_ID)."""
    import numpy as np
    hw = (place & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcc = ((place >> np.uint64(32)) & np.uint64(15)).astype(np.int64)
    nu0 = ((place >> np.uint64(40)) & np.uint64(255)).astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    dur = (en - st) / 100.0
    t0 = st.min()
    end = (en - t0) / 100.0
    start = (st - t0) / 100.0
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    simd_key = cu_key * 4 + simd
    out = {"n_cus_used": int(len(np.unique(cu_key))), "n_simds_used": int(len(np.unique(simd_key))),
           "games_per_simd": np.bincount(np.bincount(simd_key)).tolist(),
           "games_per_cu": np.bincount(np.bincount(cu_key)).tolist()}
    for lo, hi in ((0, 16), (16, 24), (24, 32), (32, 40), (40, 48), (48, 64), (64, 256)):
        sel = (nu0 >= lo) & (nu0 < hi)
        if sel.any():
            out[f"nu[{lo},{hi})"] = {"games": int(sel.sum()), "dur_mean": round(float(dur[sel].mean()), 2),
                                     "dur_max": round(float(dur[sel].max()), 2)}
    slow = np.argsort(-end)[:16]
    out["slowest_end"] = [{"g": int(i), "end": round(float(end[i]), 2), "start": round(float(start[i]), 2),
                           "dur": round(float(dur[i]), 2), "nu": int(nu0[i]),
                           "simd_mates_dur": sorted([round(float(dur[j]), 1) for j in np.nonzero(simd_key == simd_key[i])[0]])}
                          for i in slow]
    simd_sum = np.bincount(simd_key, weights=dur)
    out["simd_busy_sum_us"] = {"mean": round(float(simd_sum[simd_sum > 0].mean()), 2), "max": round(float(simd_sum.max()), 2)}
    corr = np.corrcoef(nu0, dur)[0, 1]
    out["corr_nu_dur"] = round(float(corr), 3)
    # duration vs start order
    out["corr_start_dur"] = round(float(np.corrcoef(start, dur)[0, 1]), 3)
    print(json.dumps({"tail": out}), flush=True)


def read(reset):
    buf = (ctypes.c_ulonglong * (2 * NPH))()
    _lib.check(L.mrts_phase_times(buf, reset))
    return list(buf)


for delta in (True, False):
    env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, MAP)] * (2 * E), seed=1, mask_delta=delta, source_bits=delta,
                       partial_obs=PO)
    env.reset()
    FUSED = os.environ.get("FUSED", "1") == "1" and delta
    burn = int(os.environ.get("BURNIN", 1000))
    if FUSED:
        env.random_policy(SEED, 0)
    for k in range(burn):
        if FUSED:
            env.step_fused(SEED, k + 1)
        else:
            env.random_policy(SEED, k)
            env.step()
    env.synchronize()
    read(1)
    n = 100
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = 0.0
    for k in range(n):
        if not FUSED:
            env.random_policy(SEED, 5000 + k)
        s.record()
        if FUSED:
            env.step_fused(SEED, burn + 1 + k)
        else:
            env.step()
        e.record()
        e.synchronize()
        ms += s.elapsed_time(e)
    ph = read(1)
    sp = (ctypes.c_ulonglong * (11 * E))()
    _lib.check(L.mrts_phase_spans(sp, E))
    import numpy as np
    st = np.array(sp[:E], dtype=np.float64)
    en = np.array(sp[E:2 * E], dtype=np.float64)
    place = np.array(sp[2 * E:3 * E], dtype=np.uint64)
    if os.environ.get("TAIL", "0") == "1" and delta:
        tail_report(st, en, place)
    if os.environ.get("LIB") == "span" and delta:
        # milestones (span build): us from the game's start, mean / p50 / p90 / max over games
        mnames = ["header", "loaded", "rows", "issued", "cycled", "outcome", "obs", "masks"]
        rep = {}
        prev = st
        for b, nm in enumerate(mnames):
            m = np.array(sp[(3 + b) * E:(4 + b) * E], dtype=np.float64)
            ok = m >= st
            if not ok.any():
                continue
            d = (m - st)[ok] / 100.0
            seg = (m - prev)[ok] / 100.0
            rep[nm] = {"from_start_mean": round(float(d.mean()), 2), "p90": round(float(np.percentile(d, 90)), 2),
                       "segment_mean": round(float(seg.mean()), 2)}
            prev = np.where(ok, m, prev)
        d = (en - prev) / 100.0
        rep["end"] = {"from_start_mean": round(float(((en - st) / 100.0).mean()), 2), "segment_mean": round(float(d.mean()), 2)}
        print(json.dumps({"milestones": rep}), flush=True)
    t0 = st.min()
    spans = {"dispatch_spread_us": (st.max() - t0) / 100.0, "kernel_span_us": (en.max() - t0) / 100.0,
             "game_us_mean": float((en - st).mean()) / 100.0, "game_us_p99": float(np.percentile(en - st, 99)) / 100.0,
             "game_us_max": float((en - st).max()) / 100.0,
             "start_us_percentiles": [float(np.percentile(st - t0, q)) / 100.0 for q in (10, 50, 90, 99)]}
    per = {NAMES[i]: round(ph[i] / (n * E)) for i in range(len(NAMES))}
    print(json.dumps({"mask_delta": delta, "fused_policy": FUSED, "k_env_us": 1e3 * ms / n, "last_launch": spans, "mean_cycles_per_game_step": per,
                      "total_cycles": sum(per.values()),
                      "max_game_cycles_over_100_steps": {NAMES[i]: ph[NPH + i] for i in range(len(NAMES))}}), flush=True)
    env.close()
