#!/usr/bin/env python3
"""What the timed window's fixed cost is made of (bench.py contract: synchronize, t0, K steps,
synchronize, t1), c3 workload after a 1000-step burn-in, medians of 15 windows:
  sync_only       t0; synchronize; t1 — the host's synchronize call with nothing in flight
  tiny_kernel     one 1-element torch fill + synchronize — launch + completion floor
  rollout0        rollout_fused(n_steps=0): the Python wrapper + ctypes call, no launch
  rollout_K       rollout_fused(K) for K in 1, 20, 200 (one multi-step launch)
  rollout_K_ev    the same bracketed by two fence-free events recorded from Python
  rollout_libev   the events recorded by the library around its launch (bench.py's form since round 3)
  raw_K           the same C call through prebuilt ctypes arguments (no wrapper checks)
Prints one JSON line per form."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import bench
    from microrts_amd import DeviceVecEnv

    SEED = 0x5EEDC0DE
    E = 4096
    if os.environ.get("SPIN") == "1":  # host waits spin instead of sleeping (hipDeviceScheduleSpin)
        hip = bench._FenceFreeEvent.runtime()
        assert hip.hipSetDevice(0) == 0 and hip.hipSetDeviceFlags(1) == 0
        print(json.dumps({"schedule": "spin"}), flush=True)
    env = DeviceVecEnv(2 * E, 0, 2000, ["maps/16x16/basesWorkers16x16.xml"] * (2 * E), seed=SEED)
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, 1000)
    k = [1000]
    torch.cuda.synchronize()
    dev = env.device
    stream = torch.cuda.current_stream(dev)

    def window(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    def report(name, fn, n=15, K=None):
        ts = [window(fn) for _ in range(n)]
        d = {"form": name, "median_us": float(np.median(ts)) * 1e6, "min_us": float(np.min(ts)) * 1e6}
        if K:
            d["K"] = K
            d["us_per_step"] = d["median_us"] / K
        print(json.dumps(d), flush=True)
        return d

    report("sync_only", lambda: None)
    x = torch.zeros(1, device=dev)
    report("tiny_kernel", lambda: x.fill_(1.0))

    def roll(K):
        def f():
            env.rollout_fused(SEED, k[0] + 1, K)
            k[0] += K
        return f

    report("rollout0", roll(0))
    ev = (bench._FenceFreeEvent(), bench._FenceFreeEvent())

    def roll_ev(K):
        def f():
            ev[0].record(stream)
            env.rollout_fused(SEED, k[0] + 1, K)
            k[0] += K
            ev[1].record(stream)
        return f

    h = env._h
    fn = h.L.mrts_rollout_fused_dev
    p = env._p
    args = [h.h, p(env.actions), p(env.players), p(env.obs), p(env.reward), p(env.done), p(env.masks), env.mask_player, SEED]
    sp = env._s(None)

    def raw(K):
        def f():
            rc = fn(*args, k[0] + 1, K, sp)
            assert rc == 0
            k[0] += K
        return f

    def roll_libev(K):  # bench.py's form: the library records the events (mrts_set_rollout_events)
        def f():
            env.rollout_fused(SEED, k[0] + 1, K)
            k[0] += K
        return f

    def report_libev(name, K, n=15):
        ts = []
        for _ in range(n):
            env.set_rollout_events(ev[0].h, ev[1].h)
            ts.append(window(roll_libev(K)))
        d = {"form": name, "K": K, "median_us": float(np.median(ts)) * 1e6, "min_us": float(np.min(ts)) * 1e6}
        d["us_per_step"] = d["median_us"] / K
        print(json.dumps(d), flush=True)

    for K in (1, 20, 200):
        report("rollout", roll(K), K=K)
        report("rollout_ev", roll_ev(K), K=K)
        report_libev("rollout_libev", K)
        report("raw", raw(K), K=K)
    assert not env.error_flags().any()
    env.close()


if __name__ == "__main__":
    main()
