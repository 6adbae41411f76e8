#!/bin/bash
# GPU-box profiling recipe (run through gpurun): headline bench, kernel-trace stats of the same
# command, and the two PMC passes (FETCH_SIZE and WRITE_SIZE need separate passes on gfx950).
# Usage: bash tools/gpu_profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
BARGS="--steps 100 --warmup 10 --burnin 1000 --no-cpu-baseline --no-compare"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $BARGS > "$OUT/stats.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $BARGS > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $BARGS > "$OUT/pmc_write.log" 2>&1 || exit $?
exit 0
