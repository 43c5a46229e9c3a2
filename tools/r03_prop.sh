#!/bin/bash
# One GPU call: the propagation GPU tests, smoke(), then kernel traces of the
# bench's propagation legs (tools/prop_profile.py at 64 and 1024 messages).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-prop}
K=${2:-propagation or smoke or spam or trace}
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
[ -z "$K" ] || step tests 900 ./tools/gpu_keepalive.sh python -u -m pytest tests -m gpu -x -q -k "$K" \
    --timeout 300 --timeout-method thread
step p64 200 rocprofv3 --kernel-trace --stats -d "$O/p64" -o kt --output-format csv -- \
    python3 tools/prop_profile.py --msgs 64 --batches 8
step p1024 200 rocprofv3 --kernel-trace --stats -d "$O/p1024" -o kt --output-format csv -- \
    python3 tools/prop_profile.py --msgs 1024 --batches 4
python3 tools/kt_top.py "$O/p64/kt_kernel_stats.csv" 16
python3 tools/kt_top.py "$O/p1024/kt_kernel_stats.csv" 16
