"""Diagnostic: step-kernel time and unit count vs. episode phase (16x16, 4096 games)."""
import sys, os, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from microrts_amd import DeviceVecEnv
E = 4096
env = DeviceVecEnv(2*E, 0, 2000, ["maps/16x16/basesWorkers16x16.xml"]*(2*E), seed=1)
env.reset()
res = []
for k in range(2100):
    env.random_policy(0x5EEDC0DE, k)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); env.step(); e.record()
    if k % 100 == 0:
        env.synchronize()
        u = np.mean([env.dump_state(i)[4] for i in range(0, 64, 2)])
        rows = float(env.masks[..., 0].sum().item()) / (2*E)
        res.append((k, s.elapsed_time(e)*1e3, u, rows, int(env.done.sum().item())))
        print(res[-1], flush=True)
