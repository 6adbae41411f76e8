"""World-size-2 gloo test of the multi-GPU path (microrts_amd/dist.py), on CPU.

Each rank steps ITS shard of self-play games (the CPU oracle stands in for the GPU kernels; both
consume the same per-slot streams), all-gathers the observations and takes the max time over
ranks.  Rank 0 checks that the gathered tensor equals ONE process running all 2*G games — i.e.
the shards are disjoint and sharding changes nothing but placement."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from microrts_amd import dist as mdist
from tests import oracle_py

G, STEPS, SEED = 3, 25, 0x5EEDC0DE
MAP = "maps/8x8/basesWorkers8x8.xml"


def _rollout(n_games, slot_id_base):
    env = oracle_py.OracleVecClient(2 * n_games, 0, 2000, [MAP] * (2 * n_games), seed=11, slot_id_base=slot_id_base)
    env.reset()
    for step in range(STEPS):
        m = env.get_masks(0)
        acts = np.stack([oracle_py.policy(m[s], SEED, slot_id_base + s, step, 0) for s in range(env.S)])
        obs, _, _ = env.step(acts)
    env.close()
    return obs


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = mdist.shard(rank, G)
    obs = torch.from_numpy(_rollout(G, sh["slot_id_base"]))
    gathered = mdist.gather_observations(obs)
    t = mdist.max_over_ranks(float(rank + 1), torch.device("cpu"))
    if rank == 0:
        q.put((gathered.numpy(), t))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0
    whole = _rollout(2 * G, 0)
    assert gathered.shape == (2, 2 * G) + whole.shape[1:]
    assert np.array_equal(gathered.reshape(whole.shape).astype(np.int32), whole)


def _gather_worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = mdist.shard(rank, G)
    env = oracle_py.OracleVecClient(2 * G, 0, 2000, [MAP] * (2 * G), seed=11, slot_id_base=sh["slot_id_base"])
    obs, _, _ = env.reset()
    pipe = mdist.ObservationGather(obs.shape, torch.device("cpu"), mode=mode)
    outs = []
    for step in range(6):
        m = env.get_masks(0)
        acts = np.stack([oracle_py.policy(m[s], SEED, sh["slot_id_base"] + s, step, 0) for s in range(env.S)])
        obs, _, _ = env.step(acts)
        r = pipe.push(torch.from_numpy(obs))
        outs.append(None if r is None else r.clone().numpy())
    pipe.wait()
    env.close()
    q.put((rank, outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["allgather", "learner"])
def test_observation_gather_pipeline(mode):
    """The double-buffered per-step exchange (all-gather, or gather to the learner rank) delivers
    every step's observations of both shards."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000 + (0 if mode == "allgather" else 50)
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = oracle_py.OracleVecClient(4 * G, 0, 2000, [MAP] * (4 * G), seed=11)
    whole.reset()
    for step in range(6):
        m = whole.get_masks(0)
        acts = np.stack([oracle_py.policy(m[s], SEED, s, step, 0) for s in range(whole.S)])
        o, _, _ = whole.step(acts)
        for rank in (0, 1):
            got = res[rank][step]
            if mode == "learner" and rank == 1:
                assert got is None
                continue
            assert np.array_equal(got.reshape(o.shape).astype(np.int32), o), f"rank {rank} step {step}"
    whole.close()


def test_launcher_gpus_2_equals_one_run(tmp_path):
    """`--gpus N` without torch.distributed.run spawns N ranks (microrts_amd.launch,
    the launcher bench.py uses), each with RANK / LOCAL_RANK / WORLD_SIZE set; the world the ranks see
    is 2, and their shards all-gathered equal one process running all 2G games."""
    import json
    import subprocess
    import sys

    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_launch_worker.py")
    out = str(tmp_path / "res")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, worker, "--gpus", "2", "--out", out], env=env, timeout=300)
    assert r.returncode == 0
    info = json.load(open(out + ".json"))
    assert info["n_gpus"] == 2 and info["world_size"] == 2 and info["max_time"] == 2.0
    from tests.dist_launch_worker import G as WG, rollout

    gathered = np.load(out + ".npy")
    whole = rollout(2 * WG, 0)
    assert np.array_equal(gathered.reshape(whole.shape).astype(np.int32), whole)


def test_launcher_rejects_world_mismatch(tmp_path):
    """Under a launcher, --gpus must equal WORLD_SIZE (bench.py hard-fails instead of silently
    running a different world)."""
    import subprocess
    import sys

    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_launch_worker.py")
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, worker, "--gpus", "2", "--out", str(tmp_path / "x")], env=env, timeout=120,
                       capture_output=True, text=True)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
