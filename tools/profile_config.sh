#!/bin/bash
# Per-config GPU profile (run through gpurun): the bench line, rocprofv3 kernel-trace stats of the
# same command, the FETCH_SIZE and WRITE_SIZE passes (separate: TCC slots), and one SQ issue pass
# (VALU / SALU instruction counts, VALU-active and thread cycles = lane utilisation, dual-issue
# quad-cycles, wave cycles; GRBM_GUI_ACTIVE for the clock).  Summarise with tools/profile_summary.py.
# Usage: bash tools/profile_config.sh <tag> <c2|c3|c5> [extra bench args]
set -o pipefail
TAG=${1:?tag}
CFG=${2:-c3}
shift 2
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG/$CFG
mkdir -p "$OUT"
BARGS="--config $CFG --steps 100 --warmup 10 --burnin 1000 --no-cpu-baseline --no-compare --no-gather-window --no-full-contract --no-other-configs $*"
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
# the counters describe THIS library: bench.py ignores a pmc_<cfg>.json whose hash differs
python -c "from microrts_amd._lib import device_code_sha256; print(device_code_sha256())" > "$OUT/code.sha256" || exit $?
timeout -k 10 300 python bench.py $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $BARGS > "$OUT/stats.log" 2>&1 || exit $?
timeout -k 5 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $BARGS > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -k 5 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $BARGS > "$OUT/pmc_write.log" 2>&1 || exit $?
timeout -k 5 150 rocprofv3 --pmc $SQ --kernel-trace -T --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py $BARGS > "$OUT/pmc_sq.log" 2>&1 || exit $?
exit 0
