import json, os, sys, time
sys.path.insert(0, "/root/repo")
import numpy as np, torch
from microrts_amd import DeviceVecEnv
SEED = 0x5EEDC0DE
M = "maps/16x16/basesWorkers16x16.xml"
E = 4096
for G, chunk in [(1, 10), (2, 10), (2, 1), (4, 5)]:
    n = E // G
    envs, streams = [], []
    for j in range(G):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            e = DeviceVecEnv(2 * n, 0, 2000, [M] * (2 * n), seed=SEED, slot_id_base=2 * n * j)
            e.reset(); e.random_policy(SEED, 0); e.rollout_fused(SEED, 1, 1000)
        envs.append(e); streams.append(s)
    torch.cuda.synchronize()
    k = 1001
    ts = []
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for c in range(0, 200, chunk):
            for e, s in zip(envs, streams):
                with torch.cuda.stream(s):
                    e.rollout_fused(SEED, k + c, chunk)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        k += 200
    med = float(np.median(ts))
    print(json.dumps({"groups": G, "chunk": chunk, "env_steps_per_s": E * 200 / med, "us_per_step": 1e6 * med / 200}), flush=True)
    for e in envs: e.close()
