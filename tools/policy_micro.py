"""Diagnostic: policy kernel variants on a fixed mid-episode state (16x16, 4096 games)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from microrts_amd import DeviceVecEnv, _lib  # noqa: E402

E = 4096
SEED = 0x5EEDC0DE
env = DeviceVecEnv(2 * E, 0, 2000, ["maps/16x16/basesWorkers16x16.xml"] * (2 * E), seed=1)
env.reset()
for k in range(int(os.environ.get("BURNIN", 1000))):
    env.random_policy(SEED, k)
    env.step()
env.synchronize()
h = env._h


def timeit(fn, n=200):
    fn(0)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n):
        fn(i + 1)
    e.record()
    e.synchronize()
    return 1e3 * s.elapsed_time(e) / n


def delta(i):
    _lib.check(h.L.mrts_policy_dev(h.h, env._p(env.masks), env._p(env.source), SEED, i, env._p(env.actions), None))


def full_src(i):
    _lib.check(h.L.mrts_policy_invalidate(h.h))
    delta(i)


def tiled(i):
    _lib.check(h.L.mrts_policy_dev(h.h, env._p(env.masks), None, SEED, i, env._p(env.actions), None))


small = torch.zeros(16, device="cuda")
big = torch.zeros(8192 * 256 * 7, dtype=torch.int32, device="cuda")
res = {"delta_us": timeit(delta), "full_src_us": timeit(full_src), "tiled_us": timeit(tiled),
       "torch_tiny_fill_us": timeit(lambda i: small.fill_(i)), "torch_actions_zero_us": timeit(lambda i: big.zero_()),
       "candidates_per_slot": float(env.masks[..., 0].float().sum().item()) / (2 * E)}
print(json.dumps(res))
