#!/bin/bash
# Per-kernel times of the propagation workload (tools/prop_profile.py) at 64
# and 1024 messages per batch, under rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pk}
for M in 64 1024; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$M -o kt --output-format csv -- \
        python3 tools/prop_profile.py --msgs $M --batches 6 > gpurun_out/${TAG}_$M.log 2>&1 || exit $?
    tail -2 gpurun_out/${TAG}_$M.log
    python3 tools/kt_top.py gpurun_out/${TAG}_$M/kt_kernel_stats.csv
done
