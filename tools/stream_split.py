#!/usr/bin/env python3
"""Experiment: the c3 workload (4096 self-play games, 16x16) split into G handles of 4096/G games,
each stepping on its own HIP stream, so one group's kernel tail overlaps another group's head.
Window = synchronize, t0, every group enqueues K fused steps (native rollout) on its stream,
synchronize, t1 (median of 5).  Prints env-steps/s per (G, K)."""
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
    M = "maps/16x16/basesWorkers16x16.xml"
    for G in [int(x) for x in os.environ.get("GROUPS", "1,2,4").split(",")]:
        n = E // G
        envs, streams = [], []
        for j in range(G):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                e = DeviceVecEnv(2 * n, 0, 2000, [M] * (2 * n), seed=SEED, slot_id_base=2 * n * j)
                e.reset()
                e.random_policy(SEED, 0)
                e.rollout_fused(SEED, 1, 1000)
            envs.append(e)
            streams.append(s)
        torch.cuda.synchronize()
        k = 1000
        for K in (200, 20):
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for e, s in zip(envs, streams):
                    with torch.cuda.stream(s):
                        e.rollout_fused(SEED, k + 1, K)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                k += K
            med = float(np.median(ts))
            print(json.dumps({"groups": G, "K": K, "env_steps_per_s": E * K / med, "ms_per_step": 1e3 * med / K,
                              "all_ms": [round(t * 1e3, 3) for t in ts]}), flush=True)
        for e in envs:
            assert not e.error_flags().any()
            e.close()


if __name__ == "__main__":
    main()
