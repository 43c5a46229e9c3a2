#!/bin/bash
# Kernel traces of the heartbeat with the gossip exchange (cfg3 rounds,
# tools/hb_micro.py --exchange) and of the cfg5 attack round (tools/adv_micro.py)
# per-round breakdowns with tools/kt_rounds.py (forwarding hops listed per dispatch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-hbx}
O=gpurun_out/$TAG
mkdir -p "$O"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "=== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 4 "$O/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step hbx 300 rocprofv3 --kernel-trace --stats -d "$O/hbx" -o kt --output-format csv -- \
    python3 tools/hb_micro.py --exchange --settle 8 --first-tick 59 --rounds 5
python3 tools/kt_rounds.py "$O/hbx/kt_kernel_trace.csv" 30 k_gxf_pull k_gxf_mark > "$O/hbx_rounds.txt"
python3 tools/kt_top.py "$O/hbx/kt_kernel_stats.csv" 24 > "$O/hbx_top.txt"
step adv 300 rocprofv3 --kernel-trace --stats -d "$O/adv" -o kt --output-format csv -- \
    python3 tools/adv_micro.py
python3 tools/kt_rounds.py "$O/adv/kt_kernel_trace.csv" 30 k_gxf_pull k_gxf_mark > "$O/adv_rounds.txt"
cat "$O/hbx_rounds.txt" "$O/hbx_top.txt" "$O/adv_rounds.txt"
