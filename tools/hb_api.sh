#!/bin/bash
# The cfg3 heartbeat rounds (tools/hb_micro.py --exchange, the bench's ticks)
# under a kernel + HIP runtime trace: per round the wall window, kernel busy
# time, HIP API calls and the longest host gaps (tools/hb_api.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-hbapi}
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d "$O/t" -o kt --output-format csv -- \
    python3 tools/hb_micro.py --exchange --settle 8 --first-tick 59 --rounds 5 > "$O/hb.log" 2>&1 || exit $?
python3 tools/hb_api.py "$O/hb.log" "$O/t/kt_hip_api_trace.csv" "$O/t/kt_kernel_trace.csv" > "$O/api.txt"
rm -f "$O/t/kt_hip_api_trace.csv"
tail -c 5000 "$O/api.txt"
