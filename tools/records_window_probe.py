"""Diagnostic: where the records window's fixed cost goes (bench.py records_window, one rank).
c3 shape after a 1000-step burn-in; per form, medians of 15 windows of K steps: the host time until the
rollout call returns, and until torch.cuda.synchronize() returns.
  plain    env.rollout_fused(K)                     (the headline window)
  records  RecordExchange.rollout_fused(K)          (K steps' records + one in-place all-gather)"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    from microrts_amd import DeviceVecEnv
    from microrts_amd import dist as mdist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    SEED, E = 0x5EEDC0DE, 4096
    K = int(os.environ.get("K", 20))
    env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, "maps/16x16/basesWorkers16x16.xml")] * (2 * E), seed=SEED)
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, 1000)
    torch.cuda.synchronize()
    rx = mdist.RecordExchange(env, units_per_record=64)
    nxt = 1001
    rx.rollout_fused(SEED, nxt, 3)
    nxt += 3
    rx.buffer(K)
    torch.cuda.synchronize()
    out = {}
    for form in ("plain", "records", "plain", "records"):
        ret, tot = [], []
        for _ in range(15):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if form == "plain":
                env.rollout_fused(SEED, nxt, K)
            else:
                rx.rollout_fused(SEED, nxt, K)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            nxt += K
            ret.append(1e6 * (t1 - t0))
            tot.append(1e6 * (t2 - t0))
        out[form] = {"return_us": round(statistics.median(ret), 1), "window_us": round(statistics.median(tot), 1)}
        print(json.dumps({"K": K, "form": form, **out[form]}), flush=True)
    env.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
