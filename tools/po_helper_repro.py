"""Diagnostic for the c5 render helper's stale-value case: build the helper variant
(make -C microrts_amd/csrc x1 XFLAGS1=-DMRTS_NO_PO_HELPER=0) and run this with MRTS_LIB_PATH pointing at it.
The c5 shape (2048 partially observable 32x32 games, seed 7) reaches step 1000 as 999 steps + 1 single-step
launch (no helper: correct) and as 998 steps + a 2-step launch (helper renders step 1000); the two
observations differ only in game 1667's cell 566, action plane (a worker that dies in step 1000: 1 vs
4 / 5 per view).  Prints the differing slots and cells as JSON."""
import os, sys, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import torch
from microrts_amd import DeviceVecEnv
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
SEED = 0x5EEDC0DE
obs = {}
for split in [(999, 1), (998, 2)]:
    env = DeviceVecEnv(4096, 0, 2000, [os.path.join(ROOT, "maps/BWDistantResources32x32.xml")] * 4096, seed=7,
                       partial_obs=True, max_units=256)
    env.reset(); env.random_policy(SEED, 0)
    a, b = split
    env.rollout_fused(SEED, 1, a)
    env.rollout_fused(SEED, a + 1, b)
    env.synchronize()
    obs[split] = env.obs.cpu().numpy().reshape(4096, 8, -1)
    if split == (998, 2):
        st = env.dump_state(3334)
    env.close()
A, B = obs[(999, 1)], obs[(998, 2)]
bad = np.nonzero((A != B).reshape(4096, -1).any(1))[0]
out = {"slots_differing": bad.tolist()[:20], "n": int(len(bad))}
for s in bad[:4]:
    d = np.argwhere(A[s] != B[s])
    out[str(int(s))] = [[int(p), int(c), int(A[s, p, c]), int(B[s, p, c])] for p, c in d[:12]]
out["state_3334_head"] = st[:40].tolist()
print(json.dumps(out))
