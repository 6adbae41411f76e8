#!/usr/bin/env python3
"""The full-contract leg's HBM traffic (SURVEY.md §8(d) byte contract as the Java client moves it:
every mask byte rewritten, a separate policy launch reading every mask byte, one step launch per step).

  run:        python tools/full_contract_pmc.py run [--config c3] [--steps K]
              -> one JSON line (bench.full_contract_window on the config's single-GPU shard); run it under
              rocprofv3 --kernel-trace / --pmc FETCH_SIZE / --pmc WRITE_SIZE (tools/profile_full_contract.sh)
  summarize:  python tools/full_contract_pmc.py summarize gpurun_out/<tag>/fc <tag>
              -> profiles/pmc_full_contract_<cfg>.json (per-step FETCH / WRITE bytes of the timed graph
              replay's 2K dispatches, the library hash) and profiles/<tag>_full_contract_<cfg>.md

bench.py's full_contract block reports the measured traffic from that file when its hash matches the
loaded libmrts.so."""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KERNELS = ("k_env", "k_policy")


def run(a):
    import torch
    import torch.distributed as dist

    import bench
    from microrts_amd import DeviceVecEnv
    from microrts_amd import dist as mdist

    sys.argv = [sys.argv[0], "--config", a.config, "--steps", str(a.steps)]
    ba = bench.parse()  # the bench's own defaults for this config (map, shard, burn-in, UTT)
    torch.cuda.set_device(0)
    local = 0  # bench.py passes the local rank index
    E = bench.CONFIGS[a.config][1]
    sh = mdist.shard(0, E)
    r = bench.full_contract_window(ba, sh, local, 0, E, 1, mdist, torch, dist, DeviceVecEnv)
    r.update(config=a.config, steps=a.steps, games=E)
    print(json.dumps(r), flush=True)


def dispatches(path):
    """[(start, kernel, {counter: value})] of the k_env / k_policy dispatches, in start order."""
    vals, rows = defaultdict(lambda: defaultdict(float)), {}
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith(KERNELS):
            continue
        d = int(r["Dispatch_Id"])
        vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
        rows[d] = r
    key = (lambda d: int(rows[d]["Start_Timestamp"])) if rows and "Start_Timestamp" in next(iter(rows.values())) else (lambda d: d)
    return [(key(d), rows[d]["Kernel_Name"], vals[d]) for d in sorted(rows, key=key)]


def summarize(a):
    src = a.src
    line = json.loads(open(os.path.join(src, "run.json")).read().strip().splitlines()[-1])
    K, cfg = line["steps"], line["config"]
    out = {"tag": a.tag, "config": cfg, "steps": K, "games": line["games"],
           "gfx950_code_sha256": open(os.path.join(src, "code.sha256")).read().strip()}
    per = {}
    for c, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        ds = dispatches(os.path.join(src, sub, "run_counter_collection.csv"))
        # the timed graph replay: K x (policy launch + step launch), followed by the leg's eager pass (min(K, 20)
        # policy + step pairs) and its fused variant (one policy launch, 2 warm + K fused step launches)
        tail = 2 * min(K, 20) + 1 + 2 + K
        last = ds[-2 * K - tail:-tail]
        assert len(last) == 2 * K and sum(1 for x in last if x[1].startswith("k_policy")) == K, "unexpected dispatch list"
        per[c] = sum(v[c] for _, _, v in last) * 1024 / K  # KB -> bytes, per step
        per[c + "_by_kernel"] = {n: sum(v[c] for _, k, v in last if k.startswith(n)) * 1024 / K for n in KERNELS}
    trace = list(csv.DictReader(open(os.path.join(src, "stats", "run_kernel_trace.csv"))))
    tail = 2 * min(K, 20) + 1 + 2 + K
    tr = sorted((r for r in trace if r["Kernel_Name"].startswith(KERNELS)), key=lambda r: int(r["Start_Timestamp"]))[-2 * K - tail:-tail]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr) / K / 1e3  # us per step, kernels only
    t = 2 * per["FETCH_SIZE"] + per["WRITE_SIZE"]
    out.update(fetch_size_bytes=per["FETCH_SIZE"], write_size_bytes=per["WRITE_SIZE"], traffic_bytes_per_step=t,
               by_kernel={"FETCH_SIZE": per["FETCH_SIZE_by_kernel"], "WRITE_SIZE": per["WRITE_SIZE_by_kernel"]},
               kernel_us_per_step=busy, survey_8d_bytes_per_step=line["survey_8d_bytes_per_step"],
               window_us_per_step=line["ms_per_step"] * 1e3)
    json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_full_contract_{cfg}.json"), "w"), indent=1)
    md = [f"# Full-contract leg {a.tag} — {cfg}", "", "tools/full_contract_pmc.py run (unprofiled pass):", "", "```json",
          json.dumps(line, indent=1), "```", "",
          f"Timed graph replay: {K} x (k_policy + k_env single-step, full masks); kernels {busy:.1f} us per step "
          f"(rocprofv3 kernel trace), window {line['ms_per_step'] * 1e3:.1f} us per step.", "",
          "| per step | FETCH_SIZE (x2 = bytes) | WRITE_SIZE |", "|---|---|---|"]
    for n in KERNELS:
        md.append(f"| {n} | {2 * per['FETCH_SIZE_by_kernel'][n] / 1e6:.1f} MB | {per['WRITE_SIZE_by_kernel'][n] / 1e6:.1f} MB |")
    md += ["", f"L2-fabric traffic {t / 1e6:.1f} MB per step (2 x FETCH_SIZE + WRITE_SIZE, separate --pmc passes) = "
           f"{t / (busy * 1e-6) / 1e9:.0f} GB/s over the kernels' time, {t / (line['ms_per_step'] * 1e-3) / 1e9:.0f} GB/s over "
           f"the window; SURVEY §8(d) contract bytes {line['survey_8d_bytes_per_step'] / 1e6:.1f} MB.  These are the L2's "
           "memory-side requests: Infinity-Cache (256 MiB L3) hits are counted too (MI355X_MICROARCH.md, HBM section), "
           "and the policy launch re-reads masks the step launch just wrote (165 MB < 256 MiB), so they bound HBM "
           "bytes from above — they are not a fraction of HBM peak.", ""]
    open(os.path.join(ROOT, "profiles", f"{a.tag}_full_contract_{cfg}.md"), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--config", default="c3")
    r.add_argument("--steps", type=int, default=20)
    s = sub.add_parser("summarize")
    s.add_argument("src")
    s.add_argument("tag")
    a = ap.parse_args()
    run(a) if a.cmd == "run" else summarize(a)


if __name__ == "__main__":
    main()
