#!/usr/bin/env python3
"""Experiment: the timed window's fixed cost (synchronize, t0, native rollout of K fused steps,
synchronize, t1) under HIP's device scheduling flags.  SCHED=spin|yield|blocking|default sets
hipSetDeviceFlags before the device is initialised.  c3 workload after a 1000-step burn-in; median of
9 windows per K; prints per-K medians and the fixed / per-step split of a least-squares line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hip_runtime():
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64.so" in line:
                return ctypes.CDLL(line.split()[-1])
    raise OSError("libamdhip64 not loaded")


def main():
    import numpy as np
    import torch  # loads the HIP runtime without creating the device context

    sched = os.environ.get("SCHED", "default")
    flag = {"spin": 1, "yield": 2, "blocking": 4}.get(sched)
    if flag is not None:
        rc = hip_runtime().hipSetDeviceFlags(ctypes.c_uint(flag))
        print(f"hipSetDeviceFlags({flag}) -> {rc}", file=sys.stderr)
    from microrts_amd import DeviceVecEnv

    SEED = 0x5EEDC0DE
    E = 4096
    env = DeviceVecEnv(2 * E, 0, 2000, ["maps/16x16/basesWorkers16x16.xml"] * (2 * E), seed=SEED)
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, 1000)
    k = 1001
    torch.cuda.synchronize()
    res = {}
    for K in (1, 5, 20, 100):
        ts = []
        for _ in range(9):
            env.rollout_fused(SEED, k, 5)  # warmup right before the window, as bench.py does
            k += 5
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            env.rollout_fused(SEED, k, K)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            k += K
        res[K] = float(np.median(ts)) * 1e6
    Ks = np.array(sorted(res), float)
    T = np.array([res[int(x)] for x in Ks])
    b, a = np.polyfit(Ks, T, 1)
    print(json.dumps({"sched": sched, "us_per_window": {int(x): round(res[int(x)], 1) for x in Ks},
                      "fixed_us": round(float(a), 1), "us_per_step": round(float(b), 2),
                      "k20_env_steps_per_s": E * 20 / (res[20] * 1e-6)}), flush=True)
    env.close()


if __name__ == "__main__":
    main()
