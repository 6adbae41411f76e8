#!/usr/bin/env python3
"""Diagnostic: marginal cost of each k_env phase, priced by running it twice (libmrts_ablate.so,
built with `make -C microrts_amd/csrc ablate`; g_ablate bit b doubles phase b idempotently, so the
game dynamics are unchanged).  The c3 workload is checkpointed after the burn-in; every variant
restores it, runs 5 untimed steps and times the same 100 fused steps (native rollout, HIP events);
variants are interleaved with baseline runs, 5 rounds, medians.  Prints one JSON line per phase:
the extra microseconds per step of its second copy ("SKIP x": negative = what x costs)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from microrts_amd import _lib  # noqa: E402

L = _lib.load(os.path.join(ROOT, "microrts_amd", "libmrts_ablate.so"))
L.mrts_set_ablate.argtypes = [ctypes.c_uint]
from microrts_amd import DeviceVecEnv  # noqa: E402

NAMES = ["load", "obs", "store", "maskbits", "record", "policy", "accept", "legality", "outcome+rewards", "index",
         "gone", "tables", "rank", "decode", "(issue)", "(cyclerank)", "SKIP obs", "SKIP records",
         "SKIP PO render pass", "PO render without its stores", "SKIP PO disk painting", "SKIP PO cell map",
         "SKIP PO render record", "(snapshot)"]
SEED = 0x5EEDC0DE


def main():
    import numpy as np

    E = int(os.environ.get("E", 4096))
    MAP = os.environ.get("MAP", "maps/16x16/basesWorkers16x16.xml")
    burn = int(os.environ.get("BURNIN", 1000))
    K = 100
    PO = os.environ.get("PO", "0") == "1"
    UNI = os.environ.get("UNIFORM", "0") == "1"  # c2: fused unmasked uniform rows, no masks
    env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, MAP)] * (2 * E), seed=SEED, partial_obs=PO,
                       max_units=int(os.environ.get("MAXU", 0)), with_masks=not UNI)
    roll = ((lambda first, n: env.rollout_uniform(SEED, first, n)) if UNI
            else (lambda first, n: env.rollout_fused(SEED, first, n)))
    env.reset()
    if not UNI:
        env.random_policy(SEED, 0)
    roll(1, burn)
    torch.cuda.synchronize()
    ck = env.checkpoint()
    acts = env.actions.clone()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(bits):
        assert L.mrts_set_ablate(bits) == 0
        env.restore(ck)
        env.actions.copy_(acts)
        roll(burn + 1, 5)
        s.record()
        roll(burn + 6, K)
        e.record()
        e.synchronize()
        return 1e3 * s.elapsed_time(e) / K  # us per step

    ref = run(0)
    out = {}
    default_bits = [b for b in range(len(NAMES)) if not NAMES[b].startswith("(")]
    variants = [b for b in range(len(NAMES)) if str(b) in os.environ.get("BITS", ",".join(map(str, default_bits))).split(",")]
    base, var = [], {b: [] for b in variants}
    for rnd in range(5):
        for b in variants:
            base.append(run(0))
            var[b].append(run(1 << b))
    bmed = float(np.median(base))
    print(json.dumps({"baseline_us_per_step": bmed, "spread": [round(x, 3) for x in sorted(base)], "first": ref}), flush=True)
    for b in variants:
        m = float(np.median(var[b]))
        out[NAMES[b]] = round(m - bmed, 3)
        print(json.dumps({"phase": NAMES[b], "extra_us_per_step": round(m - bmed, 3), "runs": [round(x, 3) for x in var[b]]}),
              flush=True)
    # the doubled run must leave the game exactly as the baseline does
    L.mrts_set_ablate(0)
    env.restore(ck)
    env.actions.copy_(acts)
    roll(burn + 1, 30)
    torch.cuda.synchronize()
    d0 = [env.dump_state(x) for x in range(0, 64, 2)]
    L.mrts_set_ablate((1 << 14) - 1)  # every doubling (no skips)
    env.restore(ck)
    env.actions.copy_(acts)
    roll(burn + 1, 30)
    torch.cuda.synchronize()
    d1 = [env.dump_state(x) for x in range(0, 64, 2)]
    print(json.dumps({"dynamics_unchanged": all(np.array_equal(a, b) for a, b in zip(d0, d1)), "summary": out}), flush=True)
    L.mrts_set_ablate(0)
    env.close()


if __name__ == "__main__":
    main()
