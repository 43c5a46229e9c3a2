#!/bin/bash
# Hop-kernel words-per-lane sweep (GSX_HOP_CW) at 256 and 1024 messages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for cw in ${CWS:-1 2 4}; do
  for m in ${MSGS:-256 1024}; do
    GSX_HOP_CW=$cw timeout -k 10 180 python3 tools/prop_profile.py --msgs $m --batches 3 > gpurun_out/cw_${cw}_$m.log 2>&1 || exit $?
    echo "cw=$cw m=$m $(tail -1 gpurun_out/cw_${cw}_$m.log | cut -c1-60)"
  done
done
