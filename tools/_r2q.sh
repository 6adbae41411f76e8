set -o pipefail
mkdir -p gpurun_out/r2q
timeout -k 10 300 python bench.py --config c5 > gpurun_out/r2q/c5.json 2> gpurun_out/r2q/c5.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2q/c3_k20.json 2> gpurun_out/r2q/c3_k20.err || exit $?
