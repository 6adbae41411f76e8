"""Diagnostic: k_env<MODE_STEP> time with its outputs switched off one at a time (16x16, 4096 games).

Masks for the policy come from a separate (untimed) MODE_MASKS launch when the step kernel does not
write them, so every variant plays the same games.  Prints one JSON line per variant."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from microrts_amd import DeviceVecEnv, _lib  # noqa: E402

E = int(os.environ.get("E", 4096))
MAP = os.environ.get("MAP", "maps/16x16/basesWorkers16x16.xml")
PO = os.environ.get("PO", "0") == "1"
SEED = 0x5EEDC0DE


def run(obs_on, masks_on, burnin=1000, steps=50):
    env = DeviceVecEnv(2 * E, 0, 2000, [MAP] * (2 * E), seed=1, partial_obs=PO)
    L, h = env._h.L, env._h.h
    P = env._p
    stream = torch.cuda.current_stream()
    env.reset()
    ts = []
    for k in range(burnin + steps):
        env.random_policy(SEED, k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        _lib.check(L.mrts_step_dev(h, P(env.actions), P(env.players), P(env.obs) if obs_on else None, P(env.reward),
                                   P(env.done), P(env.masks) if masks_on else None, 0, env._s(None)))
        e.record()
        if not masks_on:
            env.get_masks()
        if k >= burnin:
            ts.append((s, e))
    torch.cuda.synchronize()
    us = float(np.mean([s.elapsed_time(e) for s, e in ts])) * 1e3
    env.close()
    return us


if __name__ == "__main__":
    for obs_on, masks_on in ((True, True), (True, False), (False, True), (False, False)):
        print(json.dumps({"obs": obs_on, "masks": masks_on, "k_env_us": run(obs_on, masks_on)}), flush=True)
