set -o pipefail
# Round evidence (run through gpurun: bash tools/round_evidence.sh <tag>): parity suite, smoke, headline bench + rocprofv3 stats + PMC passes, c2 / c5 / full-mask lines
TAG=${1:-round2_a}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
bash tools/gpu_profile.sh $TAG || exit $?
for c in c2 c5; do timeout -k 10 300 python bench.py --config $c > gpurun_out/$TAG/bench_$c.json 2>gpurun_out/$TAG/bench_$c.err || exit $?; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench_k20.json 2>gpurun_out/$TAG/bench_k20.err || exit $?
timeout -k 10 300 python bench.py --mask-mode full --no-cpu-baseline > gpurun_out/$TAG/bench_fullmasks.json 2>gpurun_out/$TAG/bench_fullmasks.err || exit $?
