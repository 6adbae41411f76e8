set -o pipefail
mkdir -p gpurun_out/r2t
A="--no-cpu-baseline --no-compare"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > gpurun_out/r2t/base_$i.json 2>> gpurun_out/r2t/err.log || exit $?
  MRTS_LIB_PATH=$PWD/microrts_amd/libmrts_wt33.so timeout -k 10 300 python bench.py $A > gpurun_out/r2t/wt33_$i.json 2>> gpurun_out/r2t/err.log || exit $?
done
