set -o pipefail
mkdir -p gpurun_out/r2za
L=$PWD/microrts_amd
A="--no-cpu-baseline --no-compare"
for i in 1 2; do
  for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c $A > gpurun_out/r2za/${c}_Os_$i.json 2>> gpurun_out/r2za/err.log || exit $?
  MRTS_LIB_PATH=$L/libmrts_Oz.so timeout -k 10 300 python bench.py --config $c $A > gpurun_out/r2za/${c}_Oz_$i.json 2>> gpurun_out/r2za/err.log || exit $?
  done
done
