"""Diagnostic: where a game wave's time goes inside a multi-step launch (the bench's form), from the
timing build (make -C microrts_amd/csrc timing -> libmrts_timing.so; never loaded by the package).
The build stamps s_memtime between the step's phases and accumulates per game over the launch's
iterations; a wave waiting at a helper barrier books that wait to the phase the barrier ends.
CFG=c3|c5|c2 (bench.py's shapes), K steps after BURNIN steps; prints mean shader-clock cycles per
game-step per phase slot (kernel-body PHASE ids, then the Game methods' MPHASE ids)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from microrts_amd import _lib  # noqa: E402

L = _lib.load(os.path.join(ROOT, "microrts_amd", "libmrts_timing.so"))
L.mrts_phase_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
from microrts_amd import DeviceVecEnv  # noqa: E402

SHAPES = {"c3": ("maps/16x16/basesWorkers16x16.xml", 4096, False, 0, False),
          "c5": ("maps/BWDistantResources32x32.xml", 2048, True, 256, False),
          "c2": ("maps/8x8/basesWorkers8x8.xml", 1024, False, 0, True)}
# kernel body (k_env): 0 step head (priority, snapshot hand-off), 1 predecode, 2 decode, 3 issue,
# 4 cycle, 5 outcome / rewards / reset, 6 observation (+ helper barriers), 7 compaction, 8 mask set-up,
# 9 masks + policy, 10 end of launch; Game methods: 11-14 writeMasks / writeMasksLanes tail, 16-19 mask
# tables / bits / far attacks, 20-22 load, 23-24 decode internals
NAMES = {0: "head", 1: "predecode", 2: "decode", 3: "issue", 4: "cycle", 5: "outcome+rewards", 6: "obs+handoff",
         7: "compact", 8: "mask_setup", 9: "masks+policy", 10: "launch_end", 11: "wm11", 12: "wm12:after_bits",
         13: "wm13:record", 14: "wm14:policy", 16: "wml16:tables", 17: "wml17", 18: "wml18:bits", 19: "wml19:far",
         20: "load20", 21: "load21", 22: "load22", 23: "dec23", 24: "dec24"}
NPH = 32
SEED = 0x5EEDC0DE
cfg = os.environ.get("CFG", "c5")
mp, E, po, mu, uni = SHAPES[cfg]
K = int(os.environ.get("K", 100))
burn = int(os.environ.get("BURNIN", 1000))
env = DeviceVecEnv(2 * E, 0, 2000, [os.path.join(ROOT, mp)] * (2 * E), seed=SEED, partial_obs=po, max_units=mu,
                   with_masks=not uni)
env.reset()
if uni:
    env.rollout_uniform(SEED, 0, burn, fused=True)
else:
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, burn)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (2 * NPH))()
_lib.check(L.mrts_phase_times(buf, 1))
if uni:
    env.rollout_uniform(SEED, burn, K, fused=True)
else:
    env.rollout_fused(SEED, burn + 1, K)
torch.cuda.synchronize()
_lib.check(L.mrts_phase_times(buf, 1))
ph = list(buf)
per = {NAMES.get(i, f"p{i}"): round(ph[i] / (K * E), 1) for i in range(NPH) if ph[i]}
body = sum(ph[i] for i in range(11)) / (K * E)
print(json.dumps({"cfg": cfg, "K": K, "games": E, "cycles_per_game_step": per, "body_total": round(body, 1)}), flush=True)
