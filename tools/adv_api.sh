#!/bin/bash
# cfg5 attack rounds (tools/adv_micro.py) under a kernel + HIP runtime trace:
# per round the wall-clock window, kernel busy time, HIP API calls and host
# gaps (tools/hb_api.py), beside the per-round kernel table (tools/kt_rounds.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
export GSX_HB_WINDOWS=1
TAG=${1:-advapi}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d "$O/t" -o kt --output-format csv -- \
    python3 tools/adv_micro.py > "$O/adv.log" 2>&1 || exit $?
python3 tools/hb_api.py "$O/adv.log" "$O/t/kt_hip_api_trace.csv" "$O/t/kt_kernel_trace.csv" > "$O/api.txt"
python3 tools/kt_rounds.py "$O/t/kt_kernel_trace.csv" 30 k_gxf_pull k_gxf_mark > "$O/rounds.txt"
rm -f "$O/t/kt_hip_api_trace.csv"
head -c 6000 "$O/api.txt"
