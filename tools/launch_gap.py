#!/usr/bin/env python3
"""Diagnostic (gap build, `make -C microrts_amd/csrc gap`): where the time between two back-to-back
step launches goes.  c3 workload (E games, fused policy) after a burn-in; one native rollout of 2
launches; per launch the first wave start, the last wave end (s_memrealtime, 100 MHz) and the
gap between them; plus HIP-event time of longer rollouts for the per-step figure."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MRTS_LIB_PATH", os.path.join(ROOT, "microrts_amd", "libmrts_gap.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from microrts_amd import DeviceVecEnv, _lib  # noqa: E402

SEED = 0x5EEDC0DE


def main():
    E = int(os.environ.get("E", 4096))
    MAP = os.environ.get("MAP", "maps/16x16/basesWorkers16x16.xml")
    env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, MAP)] * (2 * E), seed=SEED)
    L = env._h.L
    L.mrts_phase_spans.argtypes = [ctypes.c_void_p, ctypes.c_int]
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, 1000)
    torch.cuda.synchronize()
    k = 1001
    out = []
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(5):
        env.rollout_fused(SEED, k, 2)
        k += 2
        torch.cuda.synchronize()
        sp = (ctypes.c_ulonglong * (11 * E))()
        _lib.check(L.mrts_phase_spans(sp, E))
        a = np.array(sp, dtype=np.float64).reshape(11, E)
        (s0, e0), (s1, e1) = (a[0], a[1]), (a[3], a[4])
        if s1.min() < s0.min():
            (s0, e0), (s1, e1) = (s1, e1), (s0, e0)
        us = lambda v: round(float(v) / 100.0, 2)  # noqa: E731
        out.append({"first_span": us(e0.max() - s0.min()), "first_spread": us(s0.max() - s0.min()),
                    "gap_last_end_to_next_first_start": us(s1.min() - e0.max()),
                    "second_span": us(e1.max() - s1.min()), "second_spread": us(s1.max() - s1.min()),
                    "game_mean": us((e1 - s1).mean()), "game_max": us((e1 - s1).max())})
        s.record()
        env.rollout_fused(SEED, k, 100)
        e.record()
        e.synchronize()
        k += 100
        out[-1]["events_us_per_step_100"] = round(1e3 * s.elapsed_time(e) / 100, 2)
    for o in out:
        print(json.dumps(o), flush=True)
    env.close()


if __name__ == "__main__":
    main()
