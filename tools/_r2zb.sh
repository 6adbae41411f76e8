set -o pipefail
mkdir -p gpurun_out/r2zb
L=$PWD/microrts_amd
A="--no-cpu-baseline --no-compare"
for i in 1 2; do
  for c in c3 c5; do
  MRTS_LIB_PATH=$L/libmrts_prev.so timeout -k 10 300 python bench.py --config $c $A > gpurun_out/r2zb/${c}_prev_$i.json 2>> gpurun_out/r2zb/err.log || exit $?
  timeout -k 10 300 python bench.py --config $c $A > gpurun_out/r2zb/${c}_hint_$i.json 2>> gpurun_out/r2zb/err.log || exit $?
  done
done
