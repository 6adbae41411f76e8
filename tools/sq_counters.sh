#!/bin/bash
# SQ instruction-mix counters of the bench command, one rocprofv3 --pmc pass per counter group
# (run through gpurun).  Usage: bash tools/sq_counters.sh <tag>; summarise with tools/sq_summary.py.
set -o pipefail
TAG=${1:-sq}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
BARGS=${SQ_BARGS:-"--steps 100 --warmup 10 --burnin 1000 --no-cpu-baseline --no-graph"}
i=0
for grp in "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -T --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $BARGS > "$OUT/p$i.log" 2>&1 || exit $?
done
exit 0
