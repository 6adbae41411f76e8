"""Golden rollouts: fixed workloads of the north-star configs, run on the CPU
oracle, recorded as one 64-bit digest per step of everything the step returns (observation, reward,
done, masks) plus the final canonical state dumps.  `make_rollout_fixtures.py` writes them to
tests/golden/rollouts/*.json; test_golden_rollouts.py re-runs the oracle against them (CPU) and
replays the same rollouts on the GPU (gpu).

Action streams are reproducible without any RNG library: masked configs use the Philox policy
(oracle_py.policy / the GPU policy kernel, bit-identical); unmasked ones use splitmix64 of
(seed, step, slot, cell, component)."""
import hashlib

import numpy as np

SEED = 0x5EEDC0DE

CONFIGS = {
    # name: map, self-play slots, bot envs, bot kind (1 = RandomBiasedAI), partial obs, policy, steps, layout
    "c2_8x8_unmasked": dict(map="maps/8x8/basesWorkers8x8.xml", n_sp=16, n_bot=0, po=False, policy="uniform", steps=300),
    "c3_16x16_masked": dict(map="maps/16x16/basesWorkers16x16.xml", n_sp=8, n_bot=0, po=False, policy="masked", steps=300),
    "c5_32x32_po_masked": dict(map="maps/BWDistantResources32x32.xml", n_sp=4, n_bot=0, po=True, policy="masked", steps=200),
    "agent_vs_randombiased_8x8": dict(map="maps/8x8/basesWorkers8x8.xml", n_sp=0, n_bot=6, po=False, policy="masked",
                                      steps=300),
    "java_rows_8x8": dict(map="maps/8x8/basesWorkers8x8.xml", n_sp=4, n_bot=2, po=False, policy="rows", steps=200),
}
BOT_ONLY = dict(map="maps/4x4/base4x4.xml", n=2, steps=500, seed=42)  # config c1: RandomBiasedAI vs RandomBiasedAI


def _mix(x):
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def splitmix_ints(seed, step, shape, highs):
    """int32 array of `shape` + (len(highs),): component k uniform-ish in [0, highs[k])."""
    idx = np.arange(int(np.prod(shape)) * len(highs), dtype=np.uint64).reshape(tuple(shape) + (len(highs),))
    with np.errstate(over="ignore"):
        x = _mix(idx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed) * np.uint64(0xD1B54A32D192ED03)
                 + np.uint64(step) * np.uint64(0x8CB92BA72F3D8DD7))
    return (x % np.asarray(highs, dtype=np.uint64)).astype(np.int32)


UNIFORM_HIGHS = [6, 4, 4, 4, 4, 7, 49]


def uniform_actions(step, S, HW):
    return splitmix_ints(SEED, step, (S, HW), UNIFORM_HIGHS)


def java_rows(step, S, HW, acts):
    """Rows [S][n][8]: every cell once (shuffled), plus HW/4 duplicate-cell rows and 2 off-map rows."""
    n_dup = HW // 4
    rows = np.zeros((S, HW + n_dup + 2, 8), np.int32)
    key = splitmix_ints(SEED ^ 0x5A5A, step, (S, HW + n_dup + 2), [1 << 30])[..., 0]
    dup_cells = splitmix_ints(SEED ^ 0x3C3C, step, (S, n_dup), [HW])[..., 0]
    dup_acts = splitmix_ints(SEED ^ 0x7777, step, (S, n_dup), UNIFORM_HIGHS)
    for s in range(S):
        r = np.concatenate([np.concatenate([np.arange(HW, dtype=np.int32)[:, None], acts[s]], axis=1),
                            np.concatenate([dup_cells[s][:, None], dup_acts[s]], axis=1),
                            np.array([[-1, 1, 1, 0, 0, 0, 0, 0], [HW + 3, 1, 0, 0, 0, 0, 0, 0]], np.int32)])
        rows[s] = r[np.argsort(key[s], kind="stable")]
    return rows


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]
