#!/usr/bin/env python3
"""Diagnostic: VALU / SALU instruction counts and VALU lane utilisation of each k_env phase, from the
SQ counters of the ablation build (libmrts_ablate.so: g_ablate bit b runs phase b a second time,
idempotently).  Run under one rocprofv3 --pmc pass:

  rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_WAVE_CYCLES --kernel-trace -T --output-format csv -d OUT -o run -- python3 tools/ablate_sq.py OUT/order.json

The workload (c3 by default; env E / MAP / PO / MAXU / UNIFORM / BURNIN as tools/ablate_price.py) is
checkpointed after the burn-in; every variant restores it and runs the same K fused steps (one
single-step launch, then one multi-step launch).  tools/ablate_sq_summary.py subtracts the baseline
launch's counters from each variant's: the counters of one extra copy of that phase.  Instruction
counts do not depend on timing, so the ablation build's larger register footprint does not matter here."""
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
from tools.ablate_price import NAMES, SEED  # noqa: E402


def main():
    E = int(os.environ.get("E", 4096))
    MAP = os.environ.get("MAP", "maps/16x16/basesWorkers16x16.xml")
    burn = int(os.environ.get("BURNIN", 1000))
    K = int(os.environ.get("K", 50))
    PO = os.environ.get("PO", "0") == "1"
    UNI = os.environ.get("UNIFORM", "0") == "1"
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
    bits = [int(b) for b in os.environ.get("BITS", ",".join(str(b) for b in range(len(NAMES)) if not NAMES[b].startswith("("))).split(",")]
    order = []
    for b in [None] + bits + [None]:
        assert L.mrts_set_ablate(0 if b is None else 1 << b) == 0
        env.restore(ck)
        env.actions.copy_(acts)
        roll(burn + 1, K)
        torch.cuda.synchronize()
        order.append("baseline" if b is None else NAMES[b])
    L.mrts_set_ablate(0)
    json.dump({"order": order, "K": K, "games": E, "steps_per_multi_launch": K - 1 if not UNI else K}, open(sys.argv[1], "w"))
    env.close()


if __name__ == "__main__":
    main()
