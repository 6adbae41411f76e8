#!/usr/bin/env python3
"""Forward-model throughput: NaiveMCTS-style playouts of `--games` clones of a root
state, `--horizon` game cycles each (MAXSIMULATIONTIME = 1024 by default), RandomBiasedAI for both
players, then SimpleSqrtEvaluationFunction3.  Prints one JSON line: game cycles/s on the GPU (HIP
events around the playout launch, state resident in HBM) and the CPU oracle's single-thread rate on a
bounded sample of the same playouts."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--map", default="maps/16x16/basesWorkers16x16.xml")
    ap.add_argument("--horizon", type=int, default=1024)
    ap.add_argument("--root-cycles", type=int, default=200, help="cycles played to make the root state")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-games", type=int, default=16)
    args = ap.parse_args()

    import numpy as np
    import torch

    from microrts_amd import ForwardModel

    fm = ForwardModel(args.games, args.map, seed=1)
    # the root: one game played for a while; every rep clones it into all games (a search's leaves)
    root = ForwardModel(1, args.map, seed=0)
    root.playout(args.root_cycles)
    root_time = int(root.dump_state(0)[0])
    restore = np.stack([np.arange(args.games), np.zeros(args.games)], 1).astype(np.int32)
    results, cyc = [], []
    for _ in range(args.reps):
        fm.copy_from(restore, src=root)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        fm.playout(args.horizon)
        ev1.record()
        torch.cuda.synchronize()
        results.append(ev0.elapsed_time(ev1))
        # cycles simulated: the time advance of a sample of games (gameovers end early)
        cyc.append(np.mean([int(fm.dump_state(g)[0]) - root_time for g in range(0, args.games, 61)]))
    ms = min(results)
    mean_cycles = float(np.mean(cyc))
    t_eval0 = torch.cuda.Event(enable_timing=True)
    t_eval1 = torch.cuda.Event(enable_timing=True)
    t_eval0.record()
    fm.evaluate(0)
    t_eval1.record()
    torch.cuda.synchronize()
    gpu_rate = args.games * mean_cycles / (ms / 1e3)

    from tests import oracle_py

    ref = oracle_py.OracleForwardModel(args.cpu_games + 1, args.map, 1, 1, seed=0)
    ref.playout(0, args.root_cycles)
    for g in range(1, args.cpu_games + 1):
        ref.copy(g, 0)
    t = time.perf_counter()
    cpu_cycles = 0
    for g in range(1, args.cpu_games + 1):
        t0 = int(ref.dump(g)[0])
        ref.playout(g, args.horizon)
        cpu_cycles += int(ref.dump(g)[0]) - t0
    cpu_s = time.perf_counter() - t
    print(json.dumps({
        "metric": "forward-model game cycles/s (NaiveMCTS.simulate, RandomBiasedAI x2)",
        "games": args.games, "map": args.map, "horizon": args.horizon, "mean_cycles_per_playout": mean_cycles,
        "playout_ms": ms, "gpu_cycles_per_s": gpu_rate, "playouts_per_s": args.games / (ms / 1e3),
        "evaluate_ms": t_eval0.elapsed_time(t_eval1),
        "cpu_baseline": {"cycles_per_s": cpu_cycles / cpu_s, "cores": 1, "kind": "port",
                         "sample": f"{args.cpu_games} playouts of the same root"},
    }))
    fm.close()
    root.close()


if __name__ == "__main__":
    main()
