#!/bin/bash
# HBM traffic of the engine's kernels from rocprofv3 PMC counters, one counter
# per pass (MI355X_MICROARCH.md: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2),
# plus the calibration kernels of tools/microbench/pmc_calib.hip.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-r01}
mkdir -p "$OUT"
make -s -C go-libp2p-pubsub_amd || exit 3
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_${C}_$TAG" -o pmc --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu --prop-steps 1 > "$OUT/pmc_${C}_$TAG.log" 2>&1
    rc=$?; echo "$C bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
    timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d "$OUT/calib_${C}_$TAG" -o calib --output-format csv -- \
        ./tools/microbench/pmc_calib > "$OUT/calib_${C}_$TAG.log" 2>&1
    rc=$?; echo "$C calib rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo pmc done
