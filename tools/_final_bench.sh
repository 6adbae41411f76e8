set -o pipefail
mkdir -p gpurun_out/r4h
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/r4h/bench_c3_k20.json 2> gpurun_out/r4h/c3k20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4h/bench_c3_k200.json 2> gpurun_out/r4h/c3k200.err || exit $?
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r4h/bench_c5_k200.json 2> gpurun_out/r4h/c5.err || exit $?
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r4h/bench_c2_k200.json 2> gpurun_out/r4h/c2.err || exit $?
timeout -k 10 300 python tests/soak_full_parity.py --config c3 --out gpurun_out/r4h/soak_c3.json > gpurun_out/r4h/soak_c3.log 2>&1 || exit $?
timeout -k 10 300 python tests/soak_full_parity.py --config c5 --out gpurun_out/r4h/soak_c5.json > gpurun_out/r4h/soak_c5.log 2>&1 || exit $?
