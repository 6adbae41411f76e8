#!/usr/bin/env python3
"""Long every-game parity soak of the shipped kernels (round 6): tests/test_full_size_every_game.py's check — every
game of c3 / c5 / c2 in the bench's form (fused masked policy or fused uniform rows, delta masks, multi-step
launches, c5's render helper wave) against oracle replicas stepping in native code — at other seeds and over a
longer horizon with launches of several lengths: 1000 + 20 + 200 + 1040 + 777 + 2000 + 63 = 5100 steps, so every
game passes max_steps (2000) at least twice (auto-resets inside launches) besides its gameovers.  At each point
every slot's observation, reward, done, masks, next action rows and state dump must equal the oracle's.

  [SOAK_SEEDS=3] [SOAK_REPEAT=2] python tools/soak_long.py [c3 c5 c2] > profiles/round6/soak_long.jsonl
  (GPU box; ~16 CPU threads for the oracle; SOAK_REPEAT repeats the launch sequence, SOAK_SEEDS runs up to three
  env seeds per config)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.chdir(ROOT)

from tests import test_full_size_every_game as T  # noqa: E402

POINTS = (1000, 20, 200, 1040, 777, 2000, 63) * int(os.environ.get("SOAK_REPEAT", "1"))
SEEDS = {"c3": (101, 211, 307), "c5": (103, 223, 311), "c2": (107, 227, 313)}
N_SEEDS = int(os.environ.get("SOAK_SEEDS", "1"))


def heartbeat():  # a progress line every 30 s (a silent GPU-box command is taken for hung after 3 minutes)
    import threading

    t0 = time.time()

    def beat():
        while True:
            time.sleep(30)
            print(f"soak_long: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def single_step_form():
    """SOAK_FORM=single: the same rollouts as one launch per step (DeviceVecEnv.set_multi_step(False): the
    single-step kernels, the gameStep(action) drop-in's form, no helper wave)"""
    from microrts_amd import DeviceVecEnv

    orig = DeviceVecEnv.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.set_multi_step(False)

    DeviceVecEnv.__init__ = init
    DeviceVecEnv.fused_multi_step = True  # (the harness asserts the bench's shape; the launches are single-step)
    DeviceVecEnv.multi_step_capable = True


def main():
    heartbeat()
    cfgs = sys.argv[1:] or ["c3", "c5", "c2"]
    form = os.environ.get("SOAK_FORM", "bench")
    if form == "single":
        single_step_form()
    T.POINTS = POINTS
    for cfg in cfgs:
        for seed in SEEDS[cfg][:N_SEEDS]:
            mp, E, po, mu, _, uniform = T.SHAPES[cfg]
            T.SHAPES[cfg] = (mp, E, po, mu, seed, uniform)
            t0 = time.time()
            err = None
            try:
                T._every_game(cfg)
            except AssertionError as e:
                err = str(e)[:2000]
            print(json.dumps({"config": cfg, "form": form, "map": mp, "games": E, "env_seed": seed, "points": list(POINTS),
                              "steps": sum(POINTS), "every_game_equal": err is None, "error": err,
                              "wall_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
