#!/bin/bash
# r04: GPU parity tests, then the profile recipe, then a full-mask-mode bench for comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
bash tools/gpu_profile.sh r04 || exit $?
timeout -k 10 300 python bench.py --mask-mode full --no-cpu-baseline > gpurun_out/r04/bench_full.json 2> gpurun_out/r04/bench_full.err || exit $?
