set -o pipefail
# Round evidence for the library in the tree (run through gpurun: bash tools/round_evidence.sh <tag>):
# the -m gpu suite, smoke(), the per-config profiles (bench line + rocprofv3 kernel trace + PMC passes,
# tools/profile_config.sh) of c3 / c5 / c2, the full-contract leg's PMC passes, and the bench lines
# (c3 at K = 20 with the CPU baseline and K = 200; c5, c2 at K = 200).  Then, here:
#   python tools/profile_summary.py gpurun_out/<tag>/<cfg> <tag>        (each cfg)
#   python tools/full_contract_pmc.py summarize gpurun_out/<tag>/fc_c3 <tag>
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
for c in c3 c5 c2; do bash tools/profile_config.sh $TAG $c || exit $?; done
bash tools/profile_full_contract.sh $TAG c3 || exit $?
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/$TAG/bench_c3_k20.json 2> gpurun_out/$TAG/bench_c3_k20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/bench_c3_k200.json 2> gpurun_out/$TAG/bench_c3_k200.err || exit $?
for c in c5 c2; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/$TAG/bench_${c}_k200.json 2> gpurun_out/$TAG/bench_$c.err || exit $?
done
exit 0
