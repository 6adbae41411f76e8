#!/bin/bash
# Same-box comparison of several library builds, interleaved: bash tools/ab_multi.sh <tag> "<configs>" <reps> <name=path.so>...
# Results: gpurun_out/<tag>/<config>_<name>_<rep>.json (tools/ab_summary.py prints them)
set -o pipefail
TAG=$1; CFGS=$2; REPS=$3; shift 3
mkdir -p gpurun_out/$TAG
A="--no-cpu-baseline --no-other-configs --no-compare ${AB_EXTRA:-}"
for i in $(seq 1 $REPS); do
  for c in $CFGS; do
    for nv in "$@"; do
      n=${nv%%=*}; v=${nv#*=}
      MRTS_LIB_PATH=$v timeout -k 10 300 python bench.py --config $c $A > gpurun_out/$TAG/${c}_${n}_$i.json 2>> gpurun_out/$TAG/err.log || exit $?
    done
  done
done
