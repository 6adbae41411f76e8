#!/usr/bin/env python3
"""Diagnostic: can a learner's one-hot batch render (mrts_render_records_onehot_dev) overlap
the records rollout on a second stream?  c3 workload (4096 games), records over a one-rank loopback
transport, L launches of K steps.  Times, with HIP events: the rollout alone, the renders alone (B random
slots of the 8-rank volume per step, rank stride 0, one render launch per rollout launch for its K steps), and
both with the render of launch i on a second stream waiting only for launch i (so it may run beside launch
i + 1).  Each of the three is warmed once and timed as the median of 3 passes (round 6: round 5's first B had
timed the side stream's first use — its one-time queue setup — inside the two-stream window: 3.29x at B = 1,024
against 1.22x serial).  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from microrts_amd import DeviceVecEnv  # noqa: E402

SEED = 0x5EEDC0DE
E = int(os.environ.get("E", 4096))
K = int(os.environ.get("K", 20))
L = int(os.environ.get("L", 10))
MAP = os.path.join(ROOT, "maps/16x16/basesWorkers16x16.xml")


def main():
    env = DeviceVecEnv(2 * E, 0, 2000, [MAP] * (2 * E), seed=SEED)
    S = 2 * E
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, 1000)
    assert env._h.L.mrts_exchange_init_loopback(env._h.h, 1, 0) == 0
    env.set_records(64, 0)
    recvs = [env.records_buffer(K) for _ in range(L)]
    k = 1001
    g = torch.Generator(device="cpu").manual_seed(3)
    out = {"games": E, "K": K, "launches": L}
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def rollouts(evs=None):
        nonlocal k
        offs = []
        for i in range(L):
            offs.append(env.rollout_fused_records(SEED, k, K, recvs[i]))
            k += K
            if evs is not None:
                evs[i].record(main_s)
        return offs

    offs = rollouts()  # warm
    torch.cuda.synchronize()
    for B in (1024, 2048, 4096, S):
        # per launch ONE render of K x B samples: B random slots of the 8-rank volume at each of its K steps
        sel = torch.randint(0, 8 * S, (K * B,), generator=g).to(torch.int32).cuda()
        soff = [torch.tensor([[int(offs[i][j][0]), 0] for j in range(K) for _ in range(B)], dtype=torch.int64).cuda()
                for i in range(L)]
        bufs = [env.render_records_onehot(recvs[0], 0, 0, sel, step_off=soff[0]) for _ in range(2)]
        t = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

        def renders(stream, offs, evs=None):
            with torch.cuda.stream(stream):
                for i in range(L):
                    if evs is not None:
                        stream.wait_event(evs[i])
                    env.render_records_onehot(recvs[i], 0, 0, sel, bufs[i & 1], step_off=soff[i], stream=stream)

        import statistics

        def timed(fn):
            vals = []
            for rep in range(4):  # pass 0 warms (first use of a stream / event pattern), then the median of 3
                t[0].record(main_s)
                fn()
                t[1].record(main_s)
                torch.cuda.synchronize()
                if rep:
                    vals.append(t[0].elapsed_time(t[1]) / (L * K))
            return statistics.median(vals)

        def compute_only():
            nonlocal offs
            offs = rollouts()

        t_c = timed(compute_only)
        t_r = timed(lambda: renders(main_s, offs))
        evs = [torch.cuda.Event() for _ in range(L)]

        def both():
            side.wait_event(t[0])
            offs2 = rollouts(evs)
            renders(side, offs2, evs)
            main_s.wait_stream(side)

        t_o = timed(both)
        out[str(B)] = {"compute_ms_per_step": t_c, "render_ms_per_step": t_r, "both_two_streams_ms_per_step": t_o,
                       "ratio_vs_compute": t_o / t_c, "serial_ratio": (t_c + t_r) / t_c,
                       "onehot_MB_per_step": bufs[0].numel() / K / 1e6}
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
