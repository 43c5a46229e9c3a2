#!/bin/bash
# Heartbeat kernel profiles: per-round kernel breakdown of the cfg5 attack
# rounds (tools/adv_micro.py) and of cfg3 rounds incl. the opportunistic-graft
# tick (tools/hb_micro.py), then FETCH_SIZE / WRITE_SIZE passes (one counter
# group per run) over the cfg3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-hb}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/adv" -o kt --output-format csv -- \
    python3 tools/adv_micro.py --no-spam > "$O/adv.log" 2>&1 || exit $?
python3 tools/hb_rounds.py "$O/adv/kt_kernel_trace.csv" > "$O/adv_rounds.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/cfg3" -o kt --output-format csv -- \
    python3 tools/hb_micro.py --rounds 4 --first-tick 59 > "$O/cfg3.log" 2>&1 || exit $?
python3 tools/hb_rounds.py "$O/cfg3/kt_kernel_trace.csv" > "$O/cfg3_rounds.txt"
if [ "${PMC:-1}" = 1 ]; then
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_fetch" -o pmc --output-format csv -- \
        python3 tools/hb_micro.py --rounds 4 --first-tick 59 > "$O/pmc_fetch.log" 2>&1 || exit $?
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_write" -o pmc --output-format csv -- \
        python3 tools/hb_micro.py --rounds 4 --first-tick 59 > "$O/pmc_write.log" 2>&1 || exit $?
fi
cat "$O/adv_rounds.txt" "$O/cfg3_rounds.txt"
