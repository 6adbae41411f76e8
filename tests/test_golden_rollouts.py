"""Golden rollouts (tests/golden/rollouts/*.json, written by tests/golden/make_rollout_fixtures.py
from the CPU oracle): one digest per step of observation + reward + done + masks.  The CPU test pins
the oracle against the committed fixtures; the gpu test replays the same rollouts through the C ABI
and must reproduce every digest."""
import json
import os

import numpy as np
import pytest

from tests import oracle_py
from tests.golden import rollouts as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "rollouts")
NAMES = sorted(R.CONFIGS)


def _load(name):
    with open(os.path.join(FIX, name + ".json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_fixture(name):
    from tests.golden.make_rollout_fixtures import run_oracle

    fx = _load(name)
    hashes, dumps = run_oracle(fx["config"])
    assert hashes == fx["step_digests"]
    assert dumps == fx["final_dumps"]


def test_oracle_reproduces_bot_only_fixture():
    from tests.golden.make_rollout_fixtures import run_bot_only

    fx = _load("c1_bot_only_4x4")
    hashes, dumps = run_bot_only(fx["config"])
    assert hashes == fx["step_digests"] and dumps == fx["final_dumps"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_replays_fixture(name):
    import torch

    assert torch.cuda.is_available()
    from microrts_amd import DeviceVecEnv

    fx = _load(name)
    cfg = fx["config"]
    S = cfg["n_sp"] + cfg["n_bot"]
    bots = ["RandomBiasedAI"] * cfg["n_bot"] if cfg["n_bot"] else None
    env = DeviceVecEnv(cfg["n_sp"], cfg["n_bot"], 2000, [cfg["map"]] * S, partial_obs=cfg["po"], ai2s=bots,
                       seed=fx["oracle_seed"])
    env.reset()
    env.synchronize()
    HW = env.dims[1] * env.dims[2]

    def dig():
        env.synchronize()
        return R.digest(env.obs.cpu().numpy(), env.reward.cpu().numpy(), env.done.cpu().numpy(), env.masks.cpu().numpy())

    got = [dig()]
    for step in range(cfg["steps"]):
        if cfg["policy"] == "uniform":
            env.step(torch.as_tensor(R.uniform_actions(step, S, HW), device=env.device))
        elif cfg["policy"] == "masked":
            env.random_policy(R.SEED, step)
            env.step()
        else:
            env.random_policy(R.SEED, step)
            env.synchronize()
            acts = env.actions.cpu().numpy()
            env.step_rows(torch.as_tensor(R.java_rows(step, S, HW, acts), device=env.device))
        got.append(dig())
        assert got[-1] == fx["step_digests"][step + 1], f"{name}: first divergence at step {step + 1}"
    assert [env.dump_state(s).tolist() for s in range(S)] == fx["final_dumps"]
    env.close()


@pytest.mark.gpu
def test_gpu_replays_bot_only_fixture():
    import torch

    assert torch.cuda.is_available()
    from microrts_amd import DeviceVecEnv

    fx = _load("c1_bot_only_4x4")
    cfg = fx["config"]
    n = cfg["n"]
    env = DeviceVecEnv(0, n, 2000, [cfg["map"]] * n, ai1s=["RandomBiasedAI"] * n, ai2s=["RandomBiasedAI"] * n,
                       seed=cfg["seed"])
    env.reset()
    for step in range(cfg["steps"]):
        env.step()
        env.synchronize()
        rw, dn = env.reward.cpu().numpy(), env.done.cpu().numpy()
        for e in range(n):
            d = R.digest(np.array([rw[e]]), np.array([dn[e]], np.uint8), env.dump_state(e))
            assert d == fx["step_digests"][e][step], f"env {e}: first divergence at step {step}"
    assert [env.dump_state(e).tolist() for e in range(n)] == fx["final_dumps"]
    env.close()
