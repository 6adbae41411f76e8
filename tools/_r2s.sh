set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2s
BARGS="--steps 100 --warmup 10 --burnin 1000 --no-cpu-baseline --no-compare"
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_WRITE_sum --kernel-trace -T --output-format csv -d gpurun_out/r2s/p1 -o run -- python3 bench.py $BARGS > gpurun_out/r2s/p1.log 2>&1 || exit $?
