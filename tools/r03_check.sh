#!/bin/bash
# One GPU call: the whole -m gpu suite and smoke(), then kernel traces of the
# cfg3 heartbeat with the gossip exchange (tools/hb_micro.py) and of the cfg5
# attack rounds (tools/adv_micro.py).  Every step has its own limit; the first
# failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-check}
mkdir -p "$O"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "=== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 3 "$O/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || step tests 900 ./tools/gpu_keepalive.sh python -u -m pytest tests -m gpu -x -v \
    --timeout 400 --timeout-method thread --durations=15
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step hbx 300 rocprofv3 --kernel-trace --stats -d "$O/hbx" -o kt --output-format csv -- \
    python3 tools/hb_micro.py --exchange --rounds 8
step adv 300 rocprofv3 --kernel-trace --stats -d "$O/adv" -o kt --output-format csv -- \
    python3 tools/adv_micro.py --no-spam
python3 tools/hb_rounds.py "$O/adv/kt_kernel_trace.csv" > "$O/adv_rounds.txt"
cat "$O/adv_rounds.txt"
grep tick "$O/hbx.log"
echo "check done"
