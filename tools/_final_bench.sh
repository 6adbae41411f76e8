set -o pipefail
mkdir -p gpurun_out/r4e
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/r4e/bench_c3_k20.json 2> gpurun_out/r4e/c3k20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4e/bench_c3_k200.json 2> gpurun_out/r4e/c3k200.err || exit $?
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r4e/bench_c5_k200.json 2> gpurun_out/r4e/c5.err || exit $?
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r4e/bench_c2_k200.json 2> gpurun_out/r4e/c2.err || exit $?
