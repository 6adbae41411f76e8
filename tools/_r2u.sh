set -o pipefail
mkdir -p gpurun_out/r2u
L=$PWD/microrts_amd
MRTS_LIB_PATH=$L/libmrts_wt97.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2u/tests97.log 2>&1 || exit $?
MRTS_LIB_PATH=$L/libmrts_wt161.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "po or PO or c5 or partial or kat" > gpurun_out/r2u/tests161.log 2>&1 || exit $?
A="--no-cpu-baseline --no-compare"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > gpurun_out/r2u/c3_base_$i.json 2>> gpurun_out/r2u/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_wt33.so timeout -k 10 300 python bench.py $A > gpurun_out/r2u/c3_wt33_$i.json 2>> gpurun_out/r2u/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_wt97.so timeout -k 10 300 python bench.py $A > gpurun_out/r2u/c3_wt97_$i.json 2>> gpurun_out/r2u/err.log || exit $?
  timeout -k 10 300 python bench.py --config c5 $A > gpurun_out/r2u/c5_base_$i.json 2>> gpurun_out/r2u/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_wt161.so timeout -k 10 300 python bench.py --config c5 $A > gpurun_out/r2u/c5_wt161_$i.json 2>> gpurun_out/r2u/err.log || exit $?
done
