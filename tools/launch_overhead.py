#!/usr/bin/env python3
"""Fixed overhead of the timed window per launch form (bench.py contract: synchronize, t0, K steps,
synchronize, t1).  For K in (20, 200) and each form — hipGraph replay of K captured fused steps,
native rollout (mrts_rollout_fused_dev: K launches from C++), Python eager step_fused calls — the
median of 7 windows on the c3 workload after a 1000-step burn-in.  Prints one JSON line per
(form, K) plus the per-step / fixed split from the K=20 / K=200 pair."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from microrts_amd import DeviceVecEnv

    SEED = 0x5EEDC0DE
    E = 4096
    env = DeviceVecEnv(2 * E, 0, 2000, ["maps/16x16/basesWorkers16x16.xml"] * (2 * E), seed=SEED)
    env.reset()
    env.random_policy(SEED, 0)
    k = 0
    env.rollout_fused(SEED, 1, 1000)
    k = 1000
    torch.cuda.synchronize()

    def window(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    res = {}
    for K in (20, 200):
        # graph
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        base = k
        with torch.cuda.graph(g, stream=cap):
            for i in range(K):
                env.step_fused(SEED, base + i + 1)
        torch.cuda.synchronize()
        k += K
        forms = {}
        ts = []
        for _ in range(7):
            ts.append(window(g.replay))
        forms["graph"] = ts
        del g

        def native():
            nonlocal k
            env.rollout_fused(SEED, k + 1, K)
            k += K

        def eager():
            nonlocal k
            for i in range(K):
                env.step_fused(SEED, k + i + 1)
            k += K

        forms["native"] = [window(native) for _ in range(7)]
        forms["eager"] = [window(eager) for _ in range(7)]
        for f, ts in forms.items():
            med = float(np.median(ts))
            res[(f, K)] = med
            print(json.dumps({"form": f, "K": K, "median_ms": med * 1e3, "ms_per_step": med * 1e3 / K,
                              "env_steps_per_s": E * K / med, "all_ms": [t * 1e3 for t in ts]}), flush=True)
    for f in ("graph", "native", "eager"):
        a, b = res[(f, 20)], res[(f, 200)]
        per = (b - a) / 180
        print(json.dumps({"form": f, "per_step_us": per * 1e6, "fixed_us": (a - 20 * per) * 1e6}), flush=True)
    assert not env.error_flags().any()
    env.close()


if __name__ == "__main__":
    main()
