#!/usr/bin/env python3
"""The host-buffer boundary's rate (PCIe-inclusive): JNIGridnetVecClient mirror, c3 size (4096 self-play
games, 16x16), numpy actions in, numpy observations / rewards / dones (and masks) out every step —
what a JNI caller handing Java arrays would see.  Not the bench value (inputs are not HBM-resident).
Actions: a fixed int32 [slots][256][7] array of uniform random components (transfer size is what
matters here; illegal rows become NONE as in Java)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from microrts_amd import JNIGridnetVecClient, UnitTypeTable  # noqa: E402


def main():
    E = int(os.environ.get("E", 4096))
    K = int(os.environ.get("K", 20))
    mp = os.path.join(ROOT, "maps/16x16/basesWorkers16x16.xml")
    vc = JNIGridnetVecClient(2 * E, 0, 2000, ["WinLossRewardFunction"], ROOT, [mp] * (2 * E), [], UnitTypeTable(), False)
    S, HW = vc.num_slots, vc.height * vc.width
    rng = np.random.default_rng(0)
    hi = np.array([6, 4, 4, 4, 4, 7, 49], np.int32)
    acts = (rng.random((S, HW, 7)) * hi).astype(np.int32)
    vc.reset([0] * S)
    for _ in range(5):
        vc.gameStep(acts)
    out = {"games": E, "slots": S, "steps": K, "action_mb": acts.nbytes / 1e6,
           "obs_mb": S * vc.num_planes * HW * 4 / 1e6, "mask_u8_mb": S * HW * vc.mask_slots / 1e6}
    for name, masks, copy in (("gameStep", None, True), ("gameStep+getMasks_u8", np.uint8, True),
                              ("gameStep+getMasks_u8_view", np.uint8, False), ("gameStep+getMasks_i32", np.int32, True),
                              ("gameStep+getMasks_i32_view", np.int32, False)):
        t0 = time.perf_counter()
        for _ in range(K):
            vc.gameStep(acts)
            if masks is not None:
                vc.getMasks(0, dtype=masks, copy=copy)
        dt = time.perf_counter() - t0
        out[name] = {"env_steps_per_s": E * K / dt, "ms_per_step": 1e3 * dt / K}
    print(json.dumps(out), flush=True)
    vc.close()


if __name__ == "__main__":
    main()
