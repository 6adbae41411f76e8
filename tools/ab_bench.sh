#!/bin/bash
# Same-box A/B of two library builds (interleaved runs): bash tools/ab_bench.sh <tag> <prev.so> "<configs>" [reps]
# Results: gpurun_out/<tag>/<config>_{prev,new}_<rep>.json
set -o pipefail
TAG=$1; PREV=$2; CFGS=${3:-c3}; REPS=${4:-2}
mkdir -p gpurun_out/$TAG
A="--no-cpu-baseline --no-other-configs ${AB_ARGS:---no-compare}"
for i in $(seq 1 $REPS); do
  for c in $CFGS; do
    MRTS_LIB_PATH=$PREV timeout -k 10 300 python bench.py --config $c $A > gpurun_out/$TAG/${c}_prev_$i.json 2>> gpurun_out/$TAG/err.log || exit $?
    timeout -k 10 300 python bench.py --config $c $A > gpurun_out/$TAG/${c}_new_$i.json 2>> gpurun_out/$TAG/err.log || exit $?
  done
done
