#!/usr/bin/env python3
"""How the host waits for the timed window's launch (bench.py: synchronize, t0, rollout, synchronize,
t1).  c3 workload (4096 games), K = 20 native multi-step rollouts; per window the wall time and the
launch's own event duration, median of N windows.  Mode (argv[1]):
  default  torch.cuda.synchronize as bench.py does
  spin     hipSetDeviceFlags(hipDeviceScheduleSpin) before the first device call
  poll     hipStreamQuery in a loop on the env's stream, then torch.cuda.synchronize
  bench    as default, with bench.py's sequence: 1000-step burn-in, a 5-step warmup launch before
           each window
The ROCclr knob ROC_ACTIVE_WAIT_TIMEOUT (µs of active wait before an interrupt wait) is set by the
caller's environment."""
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
    raise OSError("no HIP runtime mapped")


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "default"
    K = int(os.environ.get("K", "20"))
    N = int(os.environ.get("N", "25"))
    import numpy as np
    import torch

    hip = hip_runtime()
    if mode == "spin":
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))
        print(f"hipSetDeviceFlags(spin) rc={rc}", file=sys.stderr)
    from bench import _FenceFreeEvent
    from microrts_amd import DeviceVecEnv

    SEED = 0x5EEDC0DE
    E = 4096
    env = DeviceVecEnv(2 * E, 0, 2000, ["maps/16x16/basesWorkers16x16.xml"] * (2 * E), seed=SEED)
    env.reset()
    env.random_policy(SEED, 0)
    burn = 1000 if mode == "bench" else 500
    env.rollout_fused(SEED, 1, burn)
    k = burn + 1
    torch.cuda.synchronize()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
    walls, launches, polls = [], [], []
    for w in range(N + 3):
        if mode == "bench":
            env.rollout_fused(SEED, k, 5)
            k += 5
            torch.cuda.synchronize()
        ev = (_FenceFreeEvent(), _FenceFreeEvent())
        env.set_rollout_events(ev[0].h, ev[1].h)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.rollout_fused(SEED, k, K)
        n = 0
        if mode == "poll":
            while hip.hipStreamQuery(stream) != 0:
                n += 1
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        k += K
        if w >= 3:
            walls.append(t * 1e6)
            launches.append(ev[0].elapsed_time(ev[1]) * 1e3)
            polls.append(n)
    out = {"mode": mode, "K": K, "ROC_ACTIVE_WAIT_TIMEOUT": os.environ.get("ROC_ACTIVE_WAIT_TIMEOUT"),
           "window_us": float(np.median(walls)), "launch_us": float(np.median(launches)),
           "overhead_us": float(np.median(np.array(walls) - np.array(launches))),
           "window_min_max_us": [float(np.min(walls)), float(np.max(walls))], "polls": int(np.median(polls)),
           "env_steps_per_s": 2 * E * K / (np.median(walls) * 1e-6) / 2}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
