"""A bench.py-shaped program for the launcher test (tests/test_dist_gloo.py), CPU-only.

`python tests/dist_launch_worker.py --gpus N --out F` behaves like `bench.py --gpus N`: without
WORLD_SIZE it spawns N ranks through microrts_amd.launch (the bench's own launcher) and exits with
their status; each rank checks WORLD_SIZE == --gpus, joins a gloo group, steps ITS shard of
self-play games (the CPU oracle stands in for the GPU kernels: same per-slot streams), all-gathers
the observations and rank 0 writes them with the world size it saw.  Test infrastructure only.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

G, STEPS, SEED = 3, 20, 0x5EEDC0DE
MAP = "maps/8x8/basesWorkers8x8.xml"


def rollout(n_games, slot_id_base):
    import numpy as np

    from tests import oracle_py

    env = oracle_py.OracleVecClient(2 * n_games, 0, 2000, [MAP] * (2 * n_games), seed=11, slot_id_base=slot_id_base)
    env.reset()
    for step in range(STEPS):
        m = env.get_masks(0)
        acts = np.stack([oracle_py.policy(m[s], SEED, slot_id_base + s, step, 0) for s in range(env.S)])
        obs, _, _ = env.step(acts)
    env.close()
    return obs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    from microrts_amd.launch import check_world, spawn_ranks

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:], timeout=300))
    world = check_world(a.gpus)
    import numpy as np
    import torch
    import torch.distributed as dist

    from microrts_amd import dist as mdist

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    sh = mdist.shard(rank, G)
    obs = torch.from_numpy(rollout(G, sh["slot_id_base"]))
    gathered = mdist.gather_observations(obs)
    t = mdist.max_over_ranks(float(rank + 1), torch.device("cpu"))
    if rank == 0:
        np.save(a.out + ".npy", gathered.numpy())
        with open(a.out + ".json", "w") as f:
            json.dump({"n_gpus": world, "world_size": dist.get_world_size(), "max_time": t,
                       "local_rank": int(os.environ["LOCAL_RANK"])}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
