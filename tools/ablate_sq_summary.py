#!/usr/bin/env python3
"""Per-phase SQ counters from a tools/ablate_sq.py run: counters of each variant's multi-step launch
minus the baseline launch's, per game-step; VALU lane utilisation per phase.
Usage: python tools/ablate_sq_summary.py OUT  (OUT holds order.json and the rocprofv3 csv)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    src = sys.argv[1]
    meta = json.load(open(os.path.join(src, "order.json")))
    f = glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("k_env"):
            vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ds = sorted(vals)
    # every variant enqueues the same dispatch pattern (fused: a single-step launch, then the multi-step
    # one; uniform: the multi-step one): the tail of the dispatch list is len(order) groups of p; the
    # burn-in (reset, its launches) precedes them.  In each group the launch with most VALU instructions.
    n = len(meta["order"])
    p = next(q for q in (1, 2, 3) if 1 <= len(ds) - n * q <= 5)
    tail = ds[len(ds) - n * p:]
    multi = [max(tail[i * p:(i + 1) * p], key=lambda d: vals[d]["SQ_INSTS_VALU"]) for i in range(n)]
    gs = meta["games"] * meta["steps_per_multi_launch"]
    base = [vals[d] for d, n in zip(multi, meta["order"]) if n == "baseline"]
    b = {c: sum(x[c] for x in base) / len(base) for c in base[0]}
    print(f"baseline per game-step: " + ", ".join(f"{c} {b[c] / gs:.1f}" for c in sorted(b)))
    print(f"baseline lane utilisation {b['SQ_THREAD_CYCLES_VALU'] / (b['SQ_ACTIVE_INST_VALU'] * 64):.3f}")
    print("| phase | VALU | SALU | LDS | lane util | VALU thread-ops |")
    print("|---|---|---|---|---|---|")
    rows = []
    for d, n in zip(multi, meta["order"]):
        if n == "baseline":
            continue
        v = vals[d]
        dv = (v["SQ_INSTS_VALU"] - b["SQ_INSTS_VALU"]) / gs
        ds_ = (v["SQ_INSTS_SALU"] - b["SQ_INSTS_SALU"]) / gs
        dl = (v["SQ_INSTS_LDS"] - b["SQ_INSTS_LDS"]) / gs
        dt = (v["SQ_THREAD_CYCLES_VALU"] - b["SQ_THREAD_CYCLES_VALU"]) / gs
        da = (v["SQ_ACTIVE_INST_VALU"] - b["SQ_ACTIVE_INST_VALU"]) / gs
        util = dt / (da * 64) if abs(da) > 1 else float("nan")
        rows.append({"phase": n, "valu": dv, "salu": ds_, "lds": dl, "lane_util": util, "thread_ops": dt})
        print(f"| {n} | {dv:.1f} | {ds_:.1f} | {dl:.1f} | {util:.3f} | {dt:.0f} |")
    json.dump({"baseline_per_game_step": {c: b[c] / gs for c in b}, "phases": rows}, open(os.path.join(src, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
