"""One-node rank launcher for the multi-GPU env step: `bench.py --gpus N` started
without torch.distributed.run spawns its N ranks through this module.

Contract (the same environment torch.distributed.run gives each worker): RANK = LOCAL_RANK = r,
WORLD_SIZE = LOCAL_WORLD_SIZE = N, MASTER_ADDR = 127.0.0.1, MASTER_PORT = a free local port.  The
parent only forks and waits: it never imports torch or touches a GPU, so every child starts from a
clean process and selects its own device (cuda:LOCAL_RANK) before anything else.  Children share the
parent's stdout/stderr (rank 0 alone prints the JSON line).  When a rank fails, the others are
stopped (their exact PIDs) and the parent returns the first non-zero exit status.
Standard library only.
"""
import os
import signal
import socket
import subprocess
import sys
import time


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None):
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    return env


def spawn_ranks(world, cmd, timeout=None, poll=0.2):
    """Run `cmd` (argv list) as `world` ranks; returns 0 when every rank exits 0, else the first
    failing rank's status (a negative signal number becomes 128 + signal)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    port = free_port()
    procs = [subprocess.Popen(cmd, env=rank_env(r, world, port)) for r in range(world)]
    t0 = time.monotonic()
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and status == 0:
                status = bad[0] if bad[0] > 0 else 128 - bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                status = 124
                break
            time.sleep(poll)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return status


def check_world(requested):
    """Inside a launched rank: the world the launcher set must be the one the caller asked for."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != requested:
        sys.stderr.write(f"--gpus {requested} but WORLD_SIZE={world}: launch N ranks for --gpus N\n")
        raise SystemExit(2)
    return world
