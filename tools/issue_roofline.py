#!/usr/bin/env python3
"""The VALU issue ceiling of a k_env instance, from measurements, not a guessed
cycles-per-instruction constant.

Inputs:
* the issue probe's output (tools/probes/valu_issue_probe.hip, run on an MI355X): SIMD cycles per wave64
  VALU instruction per opcode class at 1 / 2 / 4 waves per SIMD, full and 8-lane EXEC;
* the kernel's ISA (`make -C microrts_amd/csrc isa` -> /tmp/mrts_kernels.s): the static histogram of its
  VALU opcodes, folded into the probe's classes.

Output (profiles/issue_ceiling_<cfg>.json, read by bench.py): per class the static share and the
measured cycles at the kernel's occupancy (c3: 4 waves per SIMD) with full EXEC, and
    c_mix = sum_i share_i * cycles_i          (cycles per VALU instruction for this mix, dense EXEC)
so the issue ceiling is 1024 SIMDs x clock / c_mix VALU instructions per second.  The static mix
stands in for the dynamic one (no counter splits VALU instructions by opcode); both are named in the
file.  The guide's figure (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles on a
SIMD-32) is reported beside it.

Usage: python tools/issue_roofline.py gpurun_out/valu_issue.jsonl /tmp/mrts_kernels.s c3
"""
import json
import os
import re
import sys
from collections import Counter

KERNELS = {  # the multi-step instance each config's bench line times
    "c3": "_ZN12_GLOBAL__N_15k_envILi0ELi16ELi320ELb0ELb1ELb0EEEvPiPKN4mrts7KStaticENS2_4KDynE",
    "c2": "_ZN12_GLOBAL__N_15k_envILi0ELi8ELi128ELb0ELb1ELb1EEEvPiPKN4mrts7KStaticENS2_4KDynE",
    "c5": "_ZN12_GLOBAL__N_15k_envILi0ELi32ELi320ELb1ELb1ELb1EEEvPiPKN4mrts7KStaticENS2_4KDynE",
}
WAVES_PER_SIMD = {"c3": 4, "c2": 1, "c5": 2}


def klass(op):
    """Probe class of a VALU opcode (the probe's op names)."""
    if op in ("v_readlane_b32", "v_writelane_b32"):
        return "v_readlane_b32"
    if op == "v_readfirstlane_b32":
        return "v_readfirstlane_b32"
    if op.startswith(("v_mul_hi", "v_mul_lo_u32", "v_mul_lo_i32", "v_mad_u64", "v_mad_i64", "v_mul_u64")):
        return "v_mul_hi_u32" if "hi" in op else "v_mul_lo_u32"
    if op.startswith(("v_mad_u32_u24", "v_mul_u32_u24", "v_mad_i32_i24", "v_mul_i32_i24")):
        return "v_mad_u32_u24"
    if op.startswith(("v_bcnt", "v_mbcnt", "v_ffbh", "v_ffbl")):
        return "v_bcnt_u32_b32"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "v_cmp_gt_u32"
    if op.startswith("v_cndmask"):
        # the SGPR-pair form (the probe's VCC-operand loop measured 16-19 cycles per instruction at any
        # occupancy, a probe artefact or hazard not seen with an SGPR pair; both are in the probe file)
        return "v_cndmask_b32_e64_sgpr"
    if op.startswith("v_bfi"):
        return "v_bfi_b32"
    if op.startswith(("v_bfe", "v_alignbit", "v_alignbyte")):
        return "v_bfe_u32"
    if op.startswith(("v_add_co", "v_addc", "v_sub_co", "v_subb", "v_subrev_co", "v_lshl_add_u64", "v_add_u64")):
        return "v_add_co_u32"
    if op.startswith(("v_max", "v_min", "v_med3")):
        return "v_max_u32"
    if op.startswith("v_mov"):
        return "v_mov_b32"
    if op.startswith(("v_sub", "v_subrev")):
        return "v_sub_u32"
    if op.startswith("v_or_b32"):
        return "v_or_b32"
    if op.startswith("v_perm"):
        return "v_perm_b32"
    if op.startswith(("v_and_or", "v_or3", "v_xad", "v_add3", "v_lshl_or", "v_lshl_add", "v_add_lshl")):
        return "v_and_or_b32"
    if op.startswith(("v_lshl", "v_lshr", "v_ashr")):
        return "v_lshlrev_b32"
    if op.startswith(("v_xor", "v_and", "v_or", "v_not")):
        return "v_xor_b32"
    return "v_add_u32"  # moves, adds, min/max, subs, conversions: full-rate integer ALU


def valu_histogram(isa_path, kernel):
    ops, on = Counter(), False
    for line in open(isa_path):
        if line.startswith(kernel + ":"):
            on = True
            continue
        if on and line.strip().startswith(".Lfunc_end"):
            break
        if not on:
            continue
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("v_") and not op.startswith(("v_mfma", "v_accvgpr")):
            ops[op] += 1
    return ops


def main():
    probe, isa, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    wps = WAVES_PER_SIMD[cfg]
    rows = [json.loads(l) for l in open(probe) if l.startswith("{")]
    cyc = {}
    cyc8 = {}
    for r in rows:
        if r["waves_per_simd"] == wps:
            (cyc if r["lanes"] == 64 else cyc8)[r["op"]] = r["cycles_per_inst_per_simd"]["median"]
    ops = valu_histogram(isa, KERNELS[cfg])
    total = sum(ops.values())
    classes = Counter()
    for op, n in ops.items():
        classes[klass(op)] += n
    share = {k: v / total for k, v in classes.items()}
    c_mix = sum(share[k] * cyc[k] for k in share)
    c_mix8 = sum(share[k] * cyc8[k] for k in share)
    out = {
        "config": cfg,
        "kernel": KERNELS[cfg],
        "waves_per_simd": wps,
        "probe": os.path.relpath(probe),
        "static_valu_instructions": total,
        "classes": {k: {"static_share": share[k], "cycles_full_exec": cyc[k], "cycles_8_lanes": cyc8.get(k)}
                    for k in sorted(share, key=lambda k: -share[k])},
        "c_mix_cycles": c_mix,
        "c_mix_cycles_8_lanes": c_mix8,
        "c_guide_cycles": 2.0,
        "note": "cycles per wave64 VALU instruction per SIMD at the kernel's occupancy, dense EXEC, weighted by the "
                "kernel's static VALU opcode mix (the dynamic mix is not observable by counters); c_mix_cycles_8_lanes: "
                "the same mix with 8 active lanes",
    }
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", f"issue_ceiling_{cfg}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
