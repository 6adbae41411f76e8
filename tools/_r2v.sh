set -o pipefail
mkdir -p gpurun_out/r2v
L=$PWD/microrts_amd
MRTS_LIB_PATH=$L/libmrts_warm.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2v/tests.log 2>&1 || exit $?
A="--no-cpu-baseline --no-compare"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > gpurun_out/r2v/c3_base_$i.json 2>> gpurun_out/r2v/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_warm.so timeout -k 10 300 python bench.py $A > gpurun_out/r2v/c3_warm_$i.json 2>> gpurun_out/r2v/err.log || exit $?
  timeout -k 10 300 python bench.py --config c5 $A > gpurun_out/r2v/c5_base_$i.json 2>> gpurun_out/r2v/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_warm.so timeout -k 10 300 python bench.py --config c5 $A > gpurun_out/r2v/c5_warm_$i.json 2>> gpurun_out/r2v/err.log || exit $?
  timeout -k 10 300 python bench.py --config c2 $A > gpurun_out/r2v/c2_base_$i.json 2>> gpurun_out/r2v/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_warm.so timeout -k 10 300 python bench.py --config c2 $A > gpurun_out/r2v/c2_warm_$i.json 2>> gpurun_out/r2v/err.log || exit $?
done
