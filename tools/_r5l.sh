set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=gpurun_out/r5m; mkdir -p $T
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_full_size_every_game.py tests/test_gpu_parity.py tests/test_kats.py tests/test_golden_rollouts.py -k "po or PO or c5 or partial or golden or kat or every or attack or ranged" > $T/tests.log 2>&1 || exit $?
for i in 1 2 3; do
  for v in new x1; do
    if [ $v = new ]; then L=microrts_amd/libmrts.so; else L=microrts_amd/libmrts_x1.so; fi
    MRTS_LIB_PATH=$L timeout -k 10 240 python bench.py --config c5 --steps 200 --no-cpu-baseline --no-gather-window --no-full-contract > $T/c5_${v}_$i.json 2>> $T/err.log || exit $?
  done
done
