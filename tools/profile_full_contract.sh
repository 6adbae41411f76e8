#!/bin/bash
# The full-contract leg under rocprofv3 (run through gpurun): an unprofiled pass (its JSON line), the
# kernel trace, and the FETCH_SIZE / WRITE_SIZE passes (separate: TCC slots).  Summarise with
# python tools/full_contract_pmc.py summarize gpurun_out/<tag>/fc_<cfg> <tag>.
# Usage: bash tools/profile_full_contract.sh <tag> [c3]
set -o pipefail
TAG=${1:?tag}
CFG=${2:-c3}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG/fc_$CFG
mkdir -p "$OUT"
A="tools/full_contract_pmc.py run --config $CFG --steps 20"
python -c "from microrts_amd._lib import device_code_sha256; print(device_code_sha256())" > "$OUT/code.sha256" || exit $?
timeout -k 10 300 python $A > "$OUT/run.json" 2> "$OUT/run.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/stats" -o run -- python3 $A > "$OUT/stats.log" 2>&1 || exit $?
timeout -k 5 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $A > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -k 5 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_write" -o run -- python3 $A > "$OUT/pmc_write.log" 2>&1 || exit $?
exit 0
