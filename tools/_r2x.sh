set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2x
BARGS="--steps 100 --warmup 10 --burnin 1000 --no-cpu-baseline --no-compare"
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --kernel-trace -T --output-format csv -d gpurun_out/r2x/p1 -o run -- python3 bench.py $BARGS > gpurun_out/r2x/p1.log 2>&1 || exit $?
