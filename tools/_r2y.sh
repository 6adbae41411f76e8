set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2y
L=$PWD/microrts_amd
A="--no-cpu-baseline --no-compare"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > gpurun_out/r2y/base_$i.json 2>> gpurun_out/r2y/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_O2.so timeout -k 10 300 python bench.py $A > gpurun_out/r2y/O2_$i.json 2>> gpurun_out/r2y/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_Os.so timeout -k 10 300 python bench.py $A > gpurun_out/r2y/Os_$i.json 2>> gpurun_out/r2y/err.log || exit $?
done
BARGS="--steps 100 --warmup 10 --burnin 1000 --no-cpu-baseline --no-compare"
MRTS_LIB_PATH=$L/libmrts_Os.so timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --kernel-trace -T --output-format csv -d gpurun_out/r2y/pOs -o run -- python3 bench.py $BARGS > gpurun_out/r2y/pOs.log 2>&1 || exit $?
