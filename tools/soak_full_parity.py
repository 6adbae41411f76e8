"""Full-size parity soak (a diagnostic tool since round 6 — tests/test_full_size_every_game.py runs the same check in the driver suite):
EVERY game of the headline configuration — not the 65-game sample of test_headline_parity.py — checked
bit for bit against the trace-pinned oracle, in bench.py's form (fused masked policy, delta masks,
multi-step launches): after the 1000-step burn-in, after a K = 20 launch and after a K = 200 launch,
each slot's observation, reward, done, mask buffer, next action rows and full state dump.

The GPU run saves its snapshots; oracle replicas of all games then run on CPU worker processes (shards
of games), each comparing its shard.  Prints one JSON line.

  python tools/soak_full_parity.py [--config c3|c5] [--workers 16] [--out profiles/round4/soak_c3.json]
"""
import argparse
import json
import multiprocessing as mp
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

SEED = 0x5EEDC0DE
BURNIN = 1000
SHAPES = {"c3": ("maps/16x16/basesWorkers16x16.xml", 4096, False, 0, 5),
          "c5": ("maps/BWDistantResources32x32.xml", 2048, True, 256, 7)}
POINTS = (("burnin", BURNIN), ("k20", 20), ("k200", 200))
FIELDS = ("obs", "reward", "done", "masks", "actions")


def gpu_run(cfg, tmp, variant="bench"):
    import torch

    from microrts_amd import DeviceVecEnv

    mp_, n_games, po, mu, seed = SHAPES[cfg]
    S = 2 * n_games
    env = DeviceVecEnv(S, 0, 2000, [os.path.join(ROOT, mp_)] * S, seed=seed, partial_obs=po, max_units=mu,
                       obs_delta=variant != "nodelta")
    if variant == "single":  # one launch per step (no multi-step launch, no helper wave)
        env.set_multi_step(False)
    else:
        assert env.fused_multi_step
    env.reset()
    env.random_policy(SEED, 0)
    k = 0
    for tag, n in POINTS:
        env.rollout_fused(SEED, k + 1, n)
        k += n
        env.synchronize()
        dumps = [env.dump_state(s) for s in range(S)]
        arrs = {"obs": env.obs, "reward": env.reward, "done": env.done, "masks": env.masks, "actions": env.actions}
        for f, v in arrs.items():  # one .npy per field: the workers memory-map their shard's rows
            np.save(os.path.join(tmp, f"{tag}_{f}.npy"), v.cpu().numpy())
        np.save(os.path.join(tmp, f"{tag}_state.npy"), np.concatenate(dumps))
        np.save(os.path.join(tmp, f"{tag}_state_off.npy"), np.cumsum([0] + [len(d) for d in dumps]))
    assert not env.error_flags().any()
    env.close()
    del torch


def shard(args):
    """Oracle replicas of games [g0, g1): run to each point and compare with the GPU's snapshot."""
    cfg, tmp, g0, g1 = args
    from tests import oracle_py

    mp_, n_games, po, mu, seed = SHAPES[cfg]
    slots = list(range(2 * g0, 2 * g1))
    ref = oracle_py.OracleVecClient(len(slots), 0, 2000, [os.path.join(ROOT, mp_)] * len(slots), seed=seed, partial_obs=po)
    ref.reset()
    t = 0
    bad = {}
    detail = []

    def act(step):
        m = ref.get_masks(0)
        return m, np.stack([oracle_py.policy(m[i], SEED, s, step, 0) for i, s in enumerate(slots)])

    for tag, n in POINTS:
        for _ in range(n):
            _, a = act(t)
            ref.step(a)
            t += 1
        z = {f: np.load(os.path.join(tmp, f"{tag}_{f}.npy"), mmap_mode="r") for f in FIELDS + ("state", "state_off")}
        sl = slice(2 * g0, 2 * g1)
        m, nxt = act(t)  # the rows the launch sampled for the next step
        got = {"obs": ref.obs, "reward": ref.reward, "done": ref.done, "masks": m, "actions": nxt}
        for f in FIELDS:
            gz, rz = np.asarray(z[f][sl]).reshape(len(slots), -1), np.asarray(got[f]).reshape(len(slots), -1)
            ok = gz == rz
            nbad = int((~ok.all(axis=1)).sum())
            if nbad:
                bad[f"{tag}/{f}"] = nbad
                for i in np.nonzero(~ok.all(axis=1))[0][:4]:  # where: slot, flat index, GPU value, oracle value
                    idx = np.nonzero(~ok[i])[0]
                    detail.append({"point": tag, "field": f, "slot": int(slots[i]), "n_diff": int(len(idx)),
                                   "first": [[int(j), int(gz[i, j]), int(rz[i, j])] for j in idx[:8]]})
        off = z["state_off"]
        st = z["state"]
        nst = sum(0 if np.array_equal(st[off[s]:off[s + 1]], ref.dump(i)) else 1 for i, s in enumerate(slots))
        if nst:
            bad[f"{tag}/state"] = nst
    ref.close()
    return g1 - g0, bad, detail


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(SHAPES), default="c3")
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--out", default=None)
    ap.add_argument("--variant", choices=["bench", "nodelta", "single"], default="bench",
                    help="bench = bench.py's form; nodelta = full observation renders; single = one launch per step")
    ap.add_argument("--gpu-into", default=None, help=argparse.SUPPRESS)  # the GPU child's role
    a = ap.parse_args()
    if a.gpu_into:
        gpu_run(a.config, a.gpu_into, a.variant)
        return
    t0 = time.time()
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        # the GPU run is a child process of its own: this process never initialises the GPU, so the
        # oracle worker processes it starts next are started from a GPU-free parent
        subprocess.run([sys.executable, os.path.abspath(__file__), "--config", a.config, "--variant", a.variant,
                        "--gpu-into", tmp], check=True)
        t_gpu = time.time() - t0
        n_games = SHAPES[a.config][1]
        step = (n_games + a.workers - 1) // a.workers
        jobs = [(a.config, tmp, g, min(g + step, n_games)) for g in range(0, n_games, step)]
        with mp.get_context("spawn").Pool(len(jobs)) as pool:
            res = pool.map(shard, jobs)
    bad, detail = {}, []
    for _, b, d in res:
        detail += d
        for k, v in b.items():
            bad[k] = bad.get(k, 0) + v
    out = {"config": a.config, "variant": a.variant, "games": sum(n for n, _, _ in res), "slots": 2 * sum(n for n, _, _ in res),
           "points": [f"{tag} (+{n} steps)" for tag, n in POINTS], "fields": list(FIELDS) + ["state"],
           "mismatching_slots": bad, "bit_exact": not bad, "gpu_s": round(t_gpu, 1), "total_s": round(time.time() - t0, 1),
           "workers": len(jobs), "mismatches": detail[:16]}
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        open(a.out, "w").write(line + "\n")
    sys.exit(0 if not bad else 1)


if __name__ == "__main__":
    main()
