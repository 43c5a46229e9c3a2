#!/bin/bash
# Propagation batch-size sweep (tools/prop_profile.py at 256/512/1024 messages).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${MSGS:-256 512 1024 2048}; do
  timeout -k 10 180 python3 tools/prop_profile.py --msgs $m --batches 3 ${PROF_ARGS:-} > gpurun_out/exp1_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/exp1_$m.log
done
