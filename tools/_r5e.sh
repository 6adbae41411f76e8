set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_headline_parity.py -k "onehot or record_exchange or step_responses" > gpurun_out/r5e/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/consumer_overlap.py > gpurun_out/r5e/overlap.json 2> gpurun_out/r5e/overlap.err || exit $?
for c in c3 c5 c2; do bash tools/profile_config.sh r5e $c || exit $?; done
bash tools/profile_full_contract.sh r5e c3 || exit $?
