set -o pipefail
# round-14 evidence: parity suite, smoke, headline bench + rocprofv3 stats + PMC (tools/gpu_profile.sh), c2 / c5 / full-mask lines
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r14_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r14_smoke.log 2>&1 || exit $?
bash tools/gpu_profile.sh r14 || exit $?
for c in c2 c5; do timeout -k 10 300 python bench.py --config $c > gpurun_out/r14/bench_$c.json 2>gpurun_out/r14/bench_$c.err || exit $?; done
timeout -k 10 300 python bench.py --mask-mode full --no-cpu-baseline > gpurun_out/r14/bench_fullmasks.json 2>gpurun_out/r14/bench_fullmasks.err || exit $?
