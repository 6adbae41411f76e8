"""The oracle's native rollout loop (oref_rollout_policy, used by the full-size every-game GPU tests)
equals the Python per-step loop the other parity tests use: getMasks(0), the Philox masked-uniform row of
each slot from its own masks (or the unmasked uniform rows), gameStep — same observations, rewards,
dones, masks and states after every call."""
import numpy as np
import pytest

from tests import oracle_py

SEED = 0x5EEDC0DE


@pytest.mark.parametrize("mp,po,uniform,base", [("maps/16x16/basesWorkers16x16.xml", False, False, 0),
                                               ("maps/BWDistantResources32x32.xml", True, False, 6),
                                               ("maps/8x8/basesWorkers8x8.xml", False, True, 10)])
def test_native_rollout_matches_python_loop(mp, po, uniform, base):
    n = 6
    A = oracle_py.OracleVecClient(n, 0, 120, [mp] * n, seed=3, partial_obs=po)
    B = oracle_py.OracleVecClient(n, 0, 120, [mp] * n, seed=3, partial_obs=po)
    A.reset()
    B.reset()
    t = 0
    for k in (1, 37, 90):  # past max_steps 120: auto-resets inside a call
        for _ in range(k):
            if uniform:
                a = np.stack([oracle_py.policy_uniform(A.H, A.W, A.K, SEED, base + s, t) for s in range(n)])
            else:
                m = A.get_masks(0)
                a = np.stack([oracle_py.policy(m[s], SEED, base + s, t, 0) for s in range(n)])
            A.step(a)
            t += 1
        B.rollout_policy(k, SEED, base, t - k, uniform=uniform)
        assert np.array_equal(A.obs, B.obs) and np.array_equal(A.reward, B.reward) and np.array_equal(A.done, B.done)
        assert np.array_equal(A.get_masks(0), B.get_masks(0))
        for s in range(n):
            assert np.array_equal(A.dump(s), B.dump(s))
    A.close()
    B.close()
