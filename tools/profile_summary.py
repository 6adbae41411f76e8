"""Summarise a tools/profile_config.sh run into profiles/<tag>_<cfg>_summary.md and the per-config
counter file profiles/pmc_<cfg>.json that bench.py reads for roofline.traffic and roofline.issue.

The timed window of bench.py (K = --steps) is ONE multi-step k_env launch: the last k_env launch
longer than ten single-step launches (the eager kernel-timing pass and the probe steps follow it).
Counters of that launch are divided by K x games (per game-step) or by K (per step).

HBM traffic per step = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE
tallies 128-B read requests at 64 B).  Issue: SQ_* counters are summed over every SIMD; per
game-step = / (K x games).  SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* are quad-cycles.  Lane utilisation
= SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64) (rocprofv3's VALUUtilization).  Clock =
GRBM_GUI_ACTIVE / 8 XCDs / launch duration (the guide's DVFS note).
"""
import argparse
import csv
import json
import os
import shutil
import statistics
from collections import defaultdict

SIMDS = 256 * 4


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def k_env_launches(rows):
    by = {}
    for r in rows:
        if r["Kernel_Name"].startswith("k_env"):
            by[int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(by))] = r
    return sorted(by.values(), key=lambda r: int(r["Start_Timestamp"]))


def timed_launch(rows, k):
    rs = k_env_launches(rows)
    single = statistics.median(dur(r) for r in rs[-k:])
    longs = [(i, r) for i, r in enumerate(rs) if dur(r) > 10 * single]
    return longs[-1] if longs else (None, None)


def counters(path):
    """{dispatch: {counter: summed value}} and {dispatch: row} for k_env dispatches."""
    vals, rows = defaultdict(lambda: defaultdict(float)), {}
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("k_env"):
            continue
        d = int(r["Dispatch_Id"])
        vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
        rows[d] = r
    return vals, rows


def the_launch(path, k):
    vals, rows = counters(path)
    ds = sorted(rows, key=lambda d: int(rows[d]["Start_Timestamp"]) if "Start_Timestamp" in rows[d] else d)
    # the timed launch = the last one whose duration (when the trace columns exist) or VALU count is
    # more than ten times the median of the last k
    def size(d):
        r = rows[d]
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            return dur(r)
        return max(vals[d].values())
    med = statistics.median(size(d) for d in ds[-k:])
    big = [d for d in ds if size(d) > 10 * med]
    return (vals[big[-1]], rows[big[-1]]) if big else (None, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src", help="gpurun_out/<tag>/<cfg>")
    ap.add_argument("tag")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles")
    bench = json.load(open(os.path.join(a.src, "bench.json")))
    cfg = bench["config"]["workload"].split(":")[0]
    K = bench["steps"]
    games = bench["config"]["envs_per_gpu"]
    trace = list(csv.DictReader(open(os.path.join(a.src, "stats", "run_kernel_trace.csv"))))
    i, r = timed_launch(trace, K)
    launch_us = dur(r) / 1e3
    singles = [dur(x) / 1e3 for x in k_env_launches(trace)[-K:]]
    out = {"tag": a.tag, "config": cfg, "workload": bench["config"]["workload"], "mask_mode": bench["config"]["mask_mode"],
           "envs_per_gpu": games, "utt": bench["config"].get("utt"), "steps_per_launch": K,
           "kernel": "k_env<MODE_STEP> multi-step",
           "trace_launch_us": launch_us, "trace_us_per_step": launch_us / K, "bench_event_us_per_step": bench["step_kernel_ms"] * 1e3,
           "single_step_launch_us": statistics.mean(singles),
           # the library the counters were taken with (tools/profile_config.sh); bench.py refuses a mismatch
           "gfx950_code_sha256": open(os.path.join(a.src, "code.sha256")).read().strip()
           if os.path.exists(os.path.join(a.src, "code.sha256")) else None}
    lines = [f"# Profile {a.tag} — {cfg}", "", "bench.py line (profiled flags):", "", "```json", json.dumps(bench, indent=1), "```", "",
             "## rocprofv3 --kernel-trace --stats (every launch of the command)", "", "```",
             open(os.path.join(a.src, "stats", "run_kernel_stats.csv")).read().strip(), "```", "",
             f"Timed window = one multi-step k_env launch (#{i} in start order): {launch_us:.1f} us for {K} steps = "
             f"**{launch_us / K:.2f} us per step** (bench.py's fence-free events: {bench['step_kernel_ms'] * 1e3:.2f} us per step); "
             f"eager single-step launches {out['single_step_launch_us']:.2f} us.", ""]
    f = w = None
    for c, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        p = os.path.join(a.src, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            v, _ = the_launch(p, K)
            if v is not None:
                if c == "FETCH_SIZE":
                    f = v[c] * 1024 / K
                else:
                    w = v[c] * 1024 / K
    if f is not None and w is not None:
        t = 2 * f + w
        out.update(traffic_bytes_per_step=t, fetch_size_bytes=f, write_size_bytes=w)
        alg = bench["roofline"]["alg_bytes_per_step"]
        lines += ["## HBM (PMC, separate passes)", "",
                  f"per step: FETCH_SIZE {f / 1e6:.2f} MB (x2 = {2 * f / 1e6:.2f}), WRITE_SIZE {w / 1e6:.2f} MB -> traffic "
                  f"{t / 1e6:.2f} MB; algorithmic (step contract) {alg / 1e6:.2f} MB; ratio {t / alg:.2f}", ""]
    p = os.path.join(a.src, "pmc_sq", "run_counter_collection.csv")
    if os.path.exists(p):
        v, row = the_launch(p, K)
        if v is not None:
            gs = K * games
            per = {c: v[c] / gs for c in v if c.startswith("SQ_")}
            util = v["SQ_THREAD_CYCLES_VALU"] / (v["SQ_ACTIVE_INST_VALU"] * 64) if v.get("SQ_ACTIVE_INST_VALU") else None
            clock = v.get("GRBM_GUI_ACTIVE", 0) / 8 / (launch_us * 1e-6) / 1e9 if v.get("GRBM_GUI_ACTIVE") else None
            waves_per_simd = games / SIMDS
            out["issue"] = {"per_game_step": per, "valu_lane_utilization": util, "clock_ghz_grbm": clock,
                            "games_per_simd": waves_per_simd,
                            "valu_busy_frac": (v["SQ_ACTIVE_INST_VALU"] / SIMDS) / (v["SQ_WAVE_CYCLES"] / games)
                            if v.get("SQ_WAVE_CYCLES") else None}
            lines += ["## Issue (SQ PMC pass; per game-step = launch total / (K x games))", "", "| counter | per game-step |", "|---|---|"]
            lines += [f"| {c} | {per[c]:.1f} |" for c in sorted(per)]
            lines += ["", f"VALU lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU x 64)): {util:.3f}" if util else "",
                      f"clock from GRBM_GUI_ACTIVE / 8 / launch: {clock:.2f} GHz" if clock else "",
                      f"VALU-active fraction of a SIMD's step (ACTIVE_INST_VALU per SIMD / WAVE_CYCLES per wave): "
                      f"{out['issue']['valu_busy_frac']:.3f}" if out["issue"]["valu_busy_frac"] else ""]
    json.dump(out, open(os.path.join(dst, f"pmc_{cfg}.json"), "w"), indent=1)
    open(os.path.join(dst, f"{a.tag}_{cfg}_summary.md"), "w").write("\n".join(lines) + "\n")
    shutil.copy(os.path.join(a.src, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"{a.tag}_{cfg}_kernel_stats.csv"))
    print("\n".join(lines[-40:]))


if __name__ == "__main__":
    main()
