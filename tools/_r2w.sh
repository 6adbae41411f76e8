set -o pipefail
mkdir -p gpurun_out/r2w
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2w/tests.log 2>&1 || exit $?
A="--no-cpu-baseline --no-compare"
for c in c3 c2 c5; do timeout -k 10 300 python bench.py --config $c $A > gpurun_out/r2w/$c.json 2>> gpurun_out/r2w/err.log || exit $?; done
BITS=6 timeout -k 10 300 python -u tools/ablate_price.py > gpurun_out/r2w/price.jsonl 2> gpurun_out/r2w/price.err || exit $?
