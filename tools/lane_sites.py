#!/usr/bin/env python3
"""The cross-lane read sites of mrts_kernels.hip and why each reads only lanes that are active.

Lists every `rl()` (readlane) call and every DPP reduction / prefix-sum call site by enclosing function, with the
argument that its source lanes executed the definition it reads: the call itself runs in wave-uniform control flow
(every lane of the game's wave active — so even if the compiler sinks the source's definition next to the use, it
is computed there for every lane), and the lanes it reads hold a value defined for them.  A site in a function
without an entry below makes the script fail, so the table cannot silently fall behind the code.  The run-time
counterpart is the audit build (`make -C microrts_amd/csrc audit`, tests/test_zz_lane_audit.py).

Usage: python tools/lane_sites.py [--markdown]
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "microrts_amd", "csrc", "mrts_kernels.hip")

# function -> why its cross-lane reads are safe
WHY = {
    "wave_reduce": "helper: DPP over all 64 lanes then lane 63 — every caller below is in uniform flow; the source "
                   "value is a select defined on every lane",
    "wave_incl_sum": "helper: DPP prefix sum — callers in uniform flow with the operand defined on every lane",
    "wave_min": "wrapper of wave_reduce", "wave_sum": "wrapper of wave_reduce",
    "loadHeader": "called from load() / nextStep() in uniform flow; hv = `l < H_WORDS ? s[l] : 0` is a select on "
                  "every lane, and the lanes read (H_TIME..H_SEQ < H_WORDS) loaded their word",
    "load": "H_FWD read in uniform flow from the same header register as loadHeader",
    "baseReservations": "wave_sum of per-lane sums accumulated in a uniform `for (o0 ...)` loop (every lane adds 0 "
                        "outside the list)",
    "cellRank": "uniform loop over the candidate mask m (a ballot); c is the caller's per-lane cell, defined on every "
                "lane (decode / issue paths compute it before the candidate test)",
    "acceptChainReg": "tpos / cost / keyR / bv are defined on every lane before the uniform loops over ballots or "
                      "r < n; the readlanes sit outside the lane tests (round 5 moved the collision scan's read out "
                      "of `if (up && ...)`); bv's conditional update is on its own lane",
    "acceptChain": "general path (> 64 reservation words): k = ctz(ballot(rank == r)) in a uniform r loop; usesPos, "
                   "tpos, cost defined on every lane",
    "issueOne": "wave_min over every lane's candidate in a uniform loop",
    "buildIndex": "key (-1 or cost | player) is set for every lane in the uniform `for (o0 ...)` body before the "
                  "ballot; the walk reads only lanes of that ballot",
    "issueBatch": "uniform loops over ballots of act / mp / np lanes; s, rank, t, prm, tx, ty, ut are the caller's "
                  "per-lane values for act lanes; ntgt / pl / ncost are written inside `if (mp)` and read only from "
                  "mp (or np ⊂ mp) lanes, after the branch reconverges; the checkDup readlanes were moved out of the "
                  "lane test in round 5",
    "pickRandomBiased": "every value is wave-uniform (uniu / uni); the `idx - seen < cnt` branch is uniform; qc is "
                        "set on every lane of the uniform q0 loop (0 outside the list) before the ballot",
    "snapshot": "observer words ow defined on every lane of the uniform q0 loop; k1 / k2 come from ballot(obs)",
    "cycle": "R <= 64 branch and the loops are uniform; myseq is a select on every lane; cu / a / prm are written "
             "for lanes k < R and read only from lanes of work ⊂ {k < R}",
    "cycleLanes": "sq / cu / a / prm written for lanes l < nu under `if (l < nu)`; read only from lanes of "
                  "work = ballot(wk) ⊂ {l < nu}, in a uniform loop",
    "quadOr": "helper: DPP quad_perm OR within each quad — called by maskBitsQuads in uniform flow (outside its lane "
              "tests) with v defined on every lane (0 for lanes without a unit)",
    "maskBitsQuads": "quadOr of v0..v2, each set on every lane (0 unless the lane's quad has a unit) before the calls, in "
                     "the uniform pass loop",
    "closerMin": "wave_min of per-lane minima of a uniform `for (o ...)` loop",
    "farAttackBits": "`if (!ballot(far)) return` is uniform; the loop over the owned mask is uniform; cuLane is the "
                     "caller's unit word of every lane < nu (owned ⊂ {l < nu})",
    "writeMasksUnits": "wave_incl_sum / lane-63 read of a count defined on every lane (0 beyond the row-set words)",
    "writeMasksLanes": "as writeMasksUnits: n = popc(gone) on every lane, uniform flow",
    "balancePerm": "the last wave of an XCD class sorts in uniform flow (`if (ballot(!ok)) return` is uniform); "
                   "sum is each lane's 4-bin total",
    "k_policy_delta": "kernel level, before any divergence: every lane's popc(dirty)",
    "k_lane_audit_probe": "the audit build's negative control (reads lane 40 from a branch only lanes 0-31 take)",
    "k_evaluate": "uniform `k < n` loop inside the uniform o0 loop; c / hpv / rv are initialised on every lane "
                  "(UC_DEAD / 0) before the `o < nu` loads",
}


def sites():
    lines = open(SRC).read().split("\n")
    fn, out = None, []
    for i, l in enumerate(lines, 1):
        m = re.match(r"\s*(?:template\s*<[^>]*>\s*)?(?:static\s+)?(?:DEV|__global__)[^(]*?\b(\w+)\s*\(", l)
        if m and not l.strip().startswith("//"):
            fn = m.group(1)
            if fn == "__launch_bounds__":
                k = re.search(r"\)\s*void\s+(\w+)\s*\(", l)
                fn = k.group(1) if k else fn
        if "#define" in l or "DEV int rl(" in l or "DEV int rlAudit" in l:
            continue
        code = l.split("//")[0]
        if re.search(r"\brl\(|\bwave_(sum|min|incl_sum)\s*\(|\bwave_reduce\s*<|update_dpp\(|\bquadOr\(", code):
            out.append((i, fn, l.strip()))
    return out


def main():
    md = "--markdown" in sys.argv
    s = sites()
    missing = sorted({f for _, f, _ in s if f not in WHY})
    by = {}
    for i, f, _ in s:
        by.setdefault(f, []).append(i)
    if md:
        print("| function | lines (mrts_kernels.hip) | why the lanes read are active |")
        print("|---|---|---|")
        for f, ls in by.items():
            print(f"| `{f}` | {', '.join(map(str, ls))} | {WHY.get(f, '**MISSING**')} |")
    else:
        for i, f, t in s:
            print(f"{i:5d} {f:20s} {t[:100]}")
    if missing:
        print(f"sites in functions without a reason: {missing}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
