"""Summarise a tools/gpu_profile.sh run into profiles/<tag>_summary.md (+ copies of the raw stats).

The rocprofv3 --stats table covers every launch of the profiled command, including the untimed
burn-in (early-episode, fewer units, faster); the summary also reports the average over the last
`--window` launches = bench.py's timed window, which is what bench.py's live HIP-event number
measures.  PMC values (FETCH_SIZE / WRITE_SIZE, KB) are per launch, window averages; FETCH_SIZE is
also shown x2 (MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE under-reports wide streaming reads by 2x;
our reads are narrow, so the true value lies between the two).

Multi-step launches (bench.json `launch_ms` set): the timed window is ONE k_env launch running all
`--window` steps; it is the last k_env launch longer than ten single-step launches (the eager
per-step kernel-timing pass and the probe steps follow it).  Its duration and counters are divided by the
window's step count (per-step figures); the eager pass gives the single-step launch average.
"""
import argparse
import csv
import json
import os
import shutil
import statistics


def window(rows, name, n):
    rs = sorted((r for r in rows if r["Kernel_Name"].startswith(name)), key=lambda r: int(r["Start_Timestamp"]))
    return rs[-n:]


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def multi_launch(rows, n):
    """(index in start order, row) of the timed multi-step k_env launch: the last launch longer than ten
    single-step launches (the median of the last n: the eager kernel-timing pass and the probe steps
    follow the timed launch; the burn-in and warmup launches precede it)."""
    rs = sorted((r for r in rows if r["Kernel_Name"].startswith("k_env")), key=lambda r: int(r["Start_Timestamp"]))
    single = statistics.median(dur(r) for r in rs[-n:])
    return [(i, r) for i, r in enumerate(rs) if dur(r) > 10 * single][-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("tag")
    ap.add_argument("--window", type=int, default=100)
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    bench = json.load(open(os.path.join(a.src, "bench.json")))
    trace = list(csv.DictReader(open(os.path.join(a.src, "stats", "run_kernel_trace.csv"))))
    lines = [f"# Profile {a.tag}", "", "bench.py line (default flags):", "", "```json", json.dumps(bench, indent=1), "```", ""]
    lines += ["## rocprofv3 --kernel-trace --stats (all launches of `bench.py --steps 100 --warmup 10 --burnin 1000`)", "",
              "```", open(os.path.join(a.src, "stats", "run_kernel_stats.csv")).read().strip(), "```", ""]
    lines += [f"## Timed window (last {a.window} launches per kernel, from the kernel trace)", "",
              "| kernel | launches | avg us | min us | max us |", "|---|---|---|---|---|"]
    multi = bench.get("launch_ms") is not None
    for k in ("k_env", "k_policy"):
        w = window(trace, k, a.window)
        d = [dur(r) / 1e3 for r in w]
        if d:
            lines.append(f"| {k}{' (eager single-step pass)' if multi and k == 'k_env' else ''} | {len(d)} | "
                         f"{statistics.mean(d):.2f} | {min(d):.2f} | {max(d):.2f} |")
    if multi:
        i, r = multi_launch(trace, a.window)
        lines += ["", f"Timed window = one multi-step k_env launch (#{i} in start order): {dur(r) / 1e3:.1f} us for "
                      f"{a.window} steps = **{dur(r) / 1e3 / a.window:.2f} us per step** (bench.py's events: "
                      f"{bench['launch_ms'] * 1e3:.1f} us for its {bench['steps']} steps = {bench['step_kernel_ms'] * 1e3:.2f} us "
                      f"per step)"]
    lines += ["", "## PMC (separate passes; KB per launch, timed-window average" + ("; k_env: per step of the multi-step launch"
              if multi else "") + ")", "",
              "| kernel | FETCH_SIZE KB | FETCH_SIZE x2 KB | WRITE_SIZE KB |", "|---|---|---|---|"]
    pmc = {}
    for c, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        p = os.path.join(a.src, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            rows = list(csv.DictReader(open(p)))
            for k in ("k_env", "k_policy"):
                if multi and k == "k_env":  # the timed multi-step launch, per step
                    _, r = multi_launch(rows, a.window)
                    pmc[(k, c)] = float(r["Counter_Value"]) / a.window
                    continue
                w = window(rows, k, a.window)
                pmc[(k, c)] = statistics.mean(float(r["Counter_Value"]) for r in w) if w else float("nan")
    for k in ("k_env", "k_policy"):
        f, wr = pmc.get((k, "FETCH_SIZE"), float("nan")), pmc.get((k, "WRITE_SIZE"), float("nan"))
        lines.append(f"| {k} | {f:.0f} | {2 * f:.0f} | {wr:.0f} |")
    if ("k_env", "WRITE_SIZE") in pmc and ("k_env", "FETCH_SIZE") in pmc:
        f, wr = pmc[("k_env", "FETCH_SIZE")] * 1024, pmc[("k_env", "WRITE_SIZE")] * 1024
        t = 2 * f + wr  # MI355X_MICROARCH.md §HBM: FETCH_SIZE x2 on gfx950; WRITE_SIZE as is
        lines += ["", f"k_env HBM traffic per {'step' if multi else 'launch'}: 2 x FETCH_SIZE + WRITE_SIZE = {t / 1e6:.1f} MB "
                      f"(uncorrected FETCH + WRITE {(f + wr) / 1e6:.1f} MB; the step's narrow loads are uncalibrated, so "
                      f"the true value lies between); step-contract algorithmic bytes per launch: "
                      f"{bench['roofline'].get('alg_bytes_per_step', bench['roofline']['alg_bytes_per_launch']) / 1e6:.1f} MB per step"]
        cfg = bench.get("config", {})
        json.dump({"tag": a.tag, "kernel": "k_env<MODE_STEP>" + (" multi-step" if multi else ""), "traffic_bytes_per_step": t,
                   "fetch_size_bytes": f, "write_size_bytes": wr, "workload": cfg.get("workload"),
                   "mask_mode": cfg.get("mask_mode"), "envs_per_gpu": cfg.get("envs_per_gpu")},
                  open(os.path.join(dst, "pmc_latest.json"), "w"), indent=1)
    open(os.path.join(dst, f"{a.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    shutil.copy(os.path.join(a.src, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"{a.tag}_kernel_stats.csv"))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
