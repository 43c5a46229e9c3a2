#!/bin/bash
# Kernel trace of the propagation workload; per-hop times (tools/hop_times.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-"256 0" "256 1" "1024 0"}; do
  set -- $cfg
  tag=kt_$1_$2
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$tag -o kt --output-format csv -- \
      python3 tools/prop_profile.py --msgs $1 --track $2 --batches 2 > gpurun_out/$tag.log 2>&1 || exit $?
  echo "== $tag"; python3 tools/hop_times.py gpurun_out/$tag/kt_kernel_trace.csv
done
