"""Every game of the benchmark configurations against the CPU oracle (VERDICT r4 "next" #2).

test_headline_parity.py replays a 65-game sample of each bench shape; round 4's hand-run soak
(now tools/soak_full_parity.py) compared every game and found a bit-exactness bug the sample had missed.
These tests are that soak in the driver's `-m gpu` suite: the shipped benchmark form of c3 (4096 self-play
games on basesWorkers16x16, fused masked policy, delta masks), c5 (2048 partially observable games on
BWDistantResources32x32, max_units 256, the render helper wave) and c2 (1024 games on basesWorkers8x8,
unmasked uniform rows drawn by the step kernel), each run as ONE native rollout call per point — a
1000-step burn-in, then a K = 20 and a K = 200 multi-step launch — and at every point every slot's
observation, reward, done, mask buffer (c3 / c5), the action rows the launch left in the tensor and the
canonical state dump (units in list order, assignments in LinkedHashMap order) must equal the oracle's.

The oracle side is one OracleVecClient per shard of games, each on its own Python thread, stepping in
native code (oref_rollout_policy: getMasks, then the same Philox rows the GPU draws, then gameStep —
JNIGridnetVecClient.java:213-316), so no GPU-produced action ever enters the oracle.  UTT v1 +
CANCEL_BOTH draws no Java random numbers, so each oracle game is an exact replica of its GPU game.
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest

from tests import oracle_py

pytestmark = pytest.mark.gpu

SEED = 0x5EEDC0DE
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POINTS = (1000, 20, 200)  # burn-in, then the driver's K and the bench default, as single rollout calls
# config: map, games, partially observable, max_units, seed, uniform policy
SHAPES = {"c3": ("maps/16x16/basesWorkers16x16.xml", 4096, False, 0, 5, False),
          "c5": ("maps/BWDistantResources32x32.xml", 2048, True, 256, 7, False),
          "c2": ("maps/8x8/basesWorkers8x8.xml", 1024, False, 0, 8, True)}


def _threads():
    """The CPUs this process may use, capped by the cgroup quota (16 on the GPU box)."""
    import bench

    return min(16, bench.all_cores())


def _gpu_points(cfg):
    """The GPU rollout in the bench's form; a host snapshot of every output and every state at each point."""
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from microrts_amd import DeviceVecEnv

    mp, E, po, mu, seed, uniform = SHAPES[cfg]
    S = 2 * E
    env = DeviceVecEnv(S, 0, 2000, [mp] * S, seed=seed, partial_obs=po, max_units=mu, with_masks=not uniform)
    assert env.multi_step_capable if uniform else env.fused_multi_step, "the bench's shape must run multi-step launches"
    env.reset()
    if not uniform:
        env.random_policy(SEED, 0)
    snaps, t = [], 0
    for n in POINTS:
        if uniform:
            env.rollout_uniform(SEED, t, n, fused=True)
        else:
            env.rollout_fused(SEED, t + 1, n)  # the first launch is a single step, then multi-step launches
        t += n
        env.synchronize()
        snap = {k: getattr(env, k).cpu().numpy() for k in ("obs", "reward", "done", "actions")}
        if not uniform:
            snap["masks"] = env.masks.cpu().numpy()
        snap["state"] = [env._h.dump(s) for s in range(S)]
        snaps.append((t, snap))
    assert not env.error_flags().any()
    env.close()
    return snaps


def _shard(cfg, g0, g1, snaps):
    """Oracle replicas of games [g0, g1): run to each point, compare; -> {what: mismatching slots}, examples."""
    mp, E, po, mu, seed, uniform = SHAPES[cfg]
    slots = np.arange(2 * g0, 2 * g1)
    ref = oracle_py.OracleVecClient(len(slots), 0, 2000, [mp] * len(slots), seed=seed, partial_obs=po)
    ref.reset()
    H, W, K = ref.H, ref.W, ref.K
    bad, ex, t = {}, [], 0
    for t_end, snap in snaps:
        ref.rollout_policy(t_end - t, SEED, 2 * g0, t, uniform=uniform)
        t = t_end
        got = {"obs": ref.obs, "reward": ref.reward, "done": ref.done}
        if uniform:  # the tensor holds the rows of the launch's last step
            got["actions"] = np.stack([oracle_py.policy_uniform(H, W, K, SEED, int(s), t - 1) for s in slots])
        else:  # the masks of the last step and the rows the launch sampled from them for the next step
            m = ref.get_masks(0)
            got["masks"] = m
            got["actions"] = np.stack([oracle_py.policy(m[i], SEED, int(s), t, 0) for i, s in enumerate(slots)])
        for f, want in got.items():
            g = np.asarray(snap[f][2 * g0:2 * g1]).reshape(len(slots), -1)
            ok = (g == np.asarray(want).reshape(len(slots), -1)).all(axis=1)
            if not ok.all():
                bad[f"step {t}: {f}"] = int((~ok).sum())
                ex.append((t, f, [int(s) for s in slots[~ok][:4]]))
        nst = [int(s) for i, s in enumerate(slots) if not np.array_equal(snap["state"][s], ref.dump(i))]
        if nst:
            bad[f"step {t}: state"] = len(nst)
            ex.append((t, "state", nst[:4]))
    ref.close()
    return bad, ex


def _every_game(cfg):
    snaps = _gpu_points(cfg)
    E = SHAPES[cfg][1]
    nt = _threads()
    step = (E + nt - 1) // nt
    bad, ex = {}, []
    with cf.ThreadPoolExecutor(nt) as pool:  # the oracle steps in native code with the GIL released
        for b, e in pool.map(lambda g0: _shard(cfg, g0, min(g0 + step, E), snaps), range(0, E, step)):
            for k, v in b.items():
                bad[k] = bad.get(k, 0) + v
            ex += e
    assert not bad, f"{cfg}: mismatching slots {bad}; first cases (step, field, slots) {ex[:8]}"


def test_every_game_c3():
    """BASELINE configs[2] as bench.py times it, all 4096 games (8192 slots)."""
    _every_game("c3")


def test_every_game_c5():
    """BASELINE configs[4] per GPU, all 2048 partially observable games, with the render helper wave
    (round 4's soak found its stale-value case here)."""
    _every_game("c5")


def test_every_game_c2():
    """BASELINE configs[1] as bench.py times it, all 1024 games, unmasked uniform rows."""
    _every_game("c2")
