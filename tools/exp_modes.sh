#!/bin/bash
# Propagation hop time by accounting mode: per-hop window (bench), late (all
# duplicates in the window), no credit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${MSGS:-256 1024}; do
  for mode in "1 10000" "1 100" "0 10000"; do
    set -- $mode
    timeout -k 10 180 python3 tools/prop_profile.py --msgs $m --batches 3 --credit $1 --latency-us $2 > gpurun_out/mode.log 2>&1 || exit $?
    echo "m=$m credit=$1 lat_us=$2 $(tail -1 gpurun_out/mode.log | cut -c1-60)"
  done
done
