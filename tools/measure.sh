#!/bin/bash
# One GPU-box measurement session: the bench line, a rocprofv3 kernel-trace
# summary of the same command, the PMC byte passes (FETCH_SIZE, WRITE_SIZE,
# one per pass, plus the calibration kernels) and the one-word gather floor.
# Each GPU step has its own limit; a crash / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "=== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 3 "$OUT/$name.err"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 900 python3 bench.py
step kt 900 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py --steps 10 --no-cpu --no-dropin
for C in FETCH_SIZE WRITE_SIZE; do
    step "pmc_$C" 900 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$C" -o pmc --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu --no-dropin --prop-steps 1 --hb-steps 2 --hb-settle 2
    step "calib_$C" 120 rocprofv3 --pmc $C --kernel-trace -d "$OUT/calib_$C" -o calib --output-format csv -- \
        ./tools/microbench/pmc_calib
done
step gather 300 ./tools/microbench/gather_rows
echo "measure done"
