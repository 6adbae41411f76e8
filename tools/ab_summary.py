"""Summarise tools/ab_bench.sh output: python tools/ab_summary.py gpurun_out/<tag>"""
import glob, json, os, sys
from collections import defaultdict

d = sys.argv[1]
res = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    name = os.path.basename(f)[:-5]
    cfg, var, _ = name.rsplit("_", 2)
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    res[(cfg, var)].append((j["value"] / 1e6, j.get("step_kernel_ms", 0) * 1e3))
for (cfg, var), v in sorted(res.items()):
    print(f"{cfg:4s} {var:5s} " + "  ".join(f"{a:7.2f}M {k:6.2f}us" for a, k in v))
