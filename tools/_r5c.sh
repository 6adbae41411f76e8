set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r5c
mkdir -p $OUT/abl
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace -T --output-format csv -d $OUT/abl -o run -- python3 tools/ablate_sq.py $OUT/abl/order.json > $OUT/abl.log 2>&1 || exit $?
SQ_BARGS="--steps 100 --warmup 10 --burnin 1000 --no-cpu-baseline --no-compare --no-gather-window --no-full-contract" bash tools/sq_counters.sh r5c/sq || exit $?
