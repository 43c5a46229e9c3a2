#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile.
# Each GPU step has its own time limit; the script stops at the first step that
# crashes, aborts or times out (a plain test failure, rc 1, is reported and the
# script goes on so the bench still runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}
STEPS=${STEPS:-all}

run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 15 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping: $name ended with rc=$rc"
        exit $rc
    fi
    return 0
}

make -s -C go-libp2p-pubsub_amd && make -s -C oracle || exit 3
rocm-smi --showproductname > "$OUT/device.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"

if [[ $STEPS == all || $STEPS == *test* ]]; then
    run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
    run bench 600 python bench.py --steps 20 --warmup 5
    grep '^{' "$OUT/bench.log" > "$OUT/bench_$TAG.json" || true
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
    run rocprof_kt 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o kt --output-format csv -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu
fi
if [[ $STEPS == *pmc* ]]; then
    run rocprof_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch_$TAG" -o pmc --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu
    run rocprof_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write_$TAG" -o pmc --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu
fi
echo "all done"
