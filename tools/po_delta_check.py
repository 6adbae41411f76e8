import os, sys, time, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from microrts_amd import DeviceVecEnv
SEED = 0x5EEDC0DE
E = 2048
for od in (True, False):
    env = DeviceVecEnv(2 * E, 0, 2000, ["maps/BWDistantResources32x32.xml"] * (2 * E), seed=SEED, partial_obs=True,
                       max_units=256, obs_delta=od)
    env.reset(); env.random_policy(SEED, 0); env.rollout_fused(SEED, 1, 600); torch.cuda.synchronize()
    for multi in (True, False):
        env.set_multi_step(multi)
        env.rollout_fused(SEED, 601, 5); torch.cuda.synchronize()
        t0 = time.perf_counter(); env.rollout_fused(SEED, 606, 100); torch.cuda.synchronize(); t = time.perf_counter() - t0
        print(json.dumps({"obs_delta": od, "multi": multi, "us_per_step": round(1e6 * t / 100, 2)}), flush=True)
    env.close()
