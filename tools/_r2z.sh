set -o pipefail
mkdir -p gpurun_out/r2z
L=$PWD/microrts_amd
MRTS_LIB_PATH=$L/libmrts_Os.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2z/tests.log 2>&1 || exit $?
A="--no-cpu-baseline --no-compare"
for i in 1 2; do
  for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c $A > gpurun_out/r2z/${c}_base_$i.json 2>> gpurun_out/r2z/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_Os.so timeout -k 10 300 python bench.py --config $c $A > gpurun_out/r2z/${c}_Os_$i.json 2>> gpurun_out/r2z/err.log || exit $?
  done
done
