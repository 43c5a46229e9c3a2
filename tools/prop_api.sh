#!/bin/bash
# One 64-message propagation call's HIP API calls beside its kernels / fills
# (tools/prop_api.py) under rocprofv3 --hip-runtime-trace --kernel-trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-propapi}
mkdir -p "$O"
timeout -k 10 200 rocprofv3 --hip-runtime-trace --kernel-trace -d "$O/t" -o kt --output-format csv -- \
    python3 tools/prop_profile.py --msgs ${2:-64} --batches 3 --warmup 2 > "$O/run.log" 2>&1 || exit $?
python3 tools/prop_api.py "$O/t/kt_hip_api_trace.csv" "$O/t/kt_kernel_trace.csv" > "$O/call.txt"
rm -f "$O/t/kt_hip_api_trace.csv"
head -c 8000 "$O/call.txt"
