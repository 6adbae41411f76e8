#!/usr/bin/env python3
"""Writes tests/golden/rollouts/*.json from the CPU oracle (see rollouts.py).  Run from the repo root
after `make -C oracle`:  python tests/golden/make_rollout_fixtures.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from tests import oracle_py  # noqa: E402
from tests.golden import rollouts as R  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "rollouts")


def run_oracle(cfg):
    S = cfg["n_sp"] + cfg["n_bot"]
    ref = oracle_py.OracleVecClient(cfg["n_sp"], cfg["n_bot"], 2000, [cfg["map"]] * S, partial_obs=cfg["po"],
                                    bot_kinds=[1] * cfg["n_bot"] if cfg["n_bot"] else None, seed=7)
    obs, rew, done = ref.reset()
    HW = ref.H * ref.W
    hashes = []
    m = ref.get_masks(0)
    hashes.append(R.digest(obs, rew, done, m))
    for step in range(cfg["steps"]):
        if cfg["policy"] == "uniform":
            acts = R.uniform_actions(step, S, HW)
        else:
            acts = np.stack([oracle_py.policy(m[s], R.SEED, s, step, 0) for s in range(S)])
        if cfg["policy"] == "rows":
            obs, rew, done = ref.step_rows(R.java_rows(step, S, HW, acts))
        else:
            obs, rew, done = ref.step(acts)
        m = ref.get_masks(0)
        hashes.append(R.digest(obs, rew, done, m))
    dumps = [ref.dump(s).tolist() for s in range(S)]
    ref.close()
    return hashes, dumps


def run_bot_only(cfg):
    hashes, dumps = [], []
    for e in range(cfg["n"]):
        b = oracle_py.OracleBotClient(cfg["map"], 1, 1, seed=cfg["seed"] + e)
        h = []
        for _ in range(cfg["steps"]):
            r, d = b.step(0)
            h.append(R.digest(np.array([r]), np.array([d], np.uint8), b.dump()))
        hashes.append(h)
        dumps.append(b.dump().tolist())
        b.close()
    return hashes, dumps


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, cfg in R.CONFIGS.items():
        hashes, dumps = run_oracle(cfg)
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump({"config": cfg, "oracle_seed": 7, "step_digests": hashes, "final_dumps": dumps}, f)
        print(name, len(hashes))
    hashes, dumps = run_bot_only(R.BOT_ONLY)
    with open(os.path.join(OUT, "c1_bot_only_4x4.json"), "w") as f:
        json.dump({"config": R.BOT_ONLY, "step_digests": hashes, "final_dumps": dumps}, f)
    print("c1_bot_only_4x4", len(hashes[0]))


if __name__ == "__main__":
    main()
