#!/bin/bash
# One GPU call: the gossip-exchange GPU tests (-k selection), then a kernel
# trace of cfg3 heartbeat rounds with the exchange (tools/hb_micro.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}
K=${2:-gossip or exchange or promise}
mkdir -p "$O"
echo "=== tests $(date +%T)"
timeout -k 10 600 ./tools/gpu_keepalive.sh python -u -m pytest tests -m gpu -x -v -k "$K" \
    --timeout 400 --timeout-method thread --durations=8 > "$O/tests.log" 2>&1
rc=$?; echo "=== tests rc=$rc"; tail -n 12 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/hbx" -o kt --output-format csv -- \
    python3 tools/hb_micro.py --exchange --rounds 8 > "$O/hbx.log" 2>&1
rc=$?; echo "=== hbx rc=$rc"; grep tick "$O/hbx.log"; [ $rc -eq 0 ] || exit $rc
python3 tools/kt_top.py "$O/hbx/kt_kernel_stats.csv" 18
