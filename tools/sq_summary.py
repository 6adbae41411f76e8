"""Per-launch / per-wave averages of the SQ counters collected by tools/sq_counters.sh (last N launches
of each kernel = bench.py's timed window).  Usage: python tools/sq_summary.py gpurun_out/<tag> [N]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    src = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [(dispatch, value)]
    waves = {}
    for f in glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
            per[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
            waves[k] = int(r.get("Grid_Size", 0) or 0) // max(1, int(r.get("Workgroup_Size", 1) or 1))
    for k in sorted(per):
        if not k.startswith("k_"):
            continue
        print(f"## {k}")
        print("| counter | per launch | per wave |")
        print("|---|---|---|")
        for c in sorted(per[k]):
            # several rows per dispatch (one per XCD/SE instance): sum per dispatch
            by = defaultdict(float)
            for d, v in per[k][c]:
                by[d] += v
            vals = [by[d] for d in sorted(by)][-n:]
            avg = sum(vals) / len(vals)
            w = waves.get(k) or 1
            print(f"| {c} | {avg:.0f} | {avg / w:.1f} |")
        print()


if __name__ == "__main__":
    main()
