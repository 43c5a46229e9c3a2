#!/bin/bash
# The evidence of a round's final tree, in parts that each fit one gpurun call:
#   suite  the -m gpu suite, then the default bench line (bench.py, N = 1)
#   prof   rocprofv3 --kernel-trace --stats of the same bench command (+ the
#          per-grid split of the headline kernel), the heartbeat / cfg5 round
#          tables (tools/hbx_prof.sh) and the propagation kernel tops (prop_kt.sh)
# Outputs under gpurun_out/$TAG/ (copied into profiles/ afterwards).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
PART=$1
TAG=${2:-final}
O=gpurun_out/$TAG
mkdir -p "$O"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "=== $name $(date +%T)" >&2
    timeout -k 10 "$secs" "$@"
    local rc=$?
    echo "=== $name rc=$rc $(date +%T)" >&2
    return $rc
}
case "$PART" in
suite)
    step tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 &&
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 &&
    step bench 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
    ;;
prof)
    step kt 600 rocprofv3 --kernel-trace --stats -d "$O/kt" -o run --output-format csv -- python3 bench.py \
        > "$O/kt_bench.json" 2> "$O/kt_bench.err" &&
    python3 tools/kt_split.py "$O/kt/run_kernel_trace.csv" > "$O/kernel_stats_by_grid.csv" 2> /dev/null
    step hbx 400 bash tools/hbx_prof.sh "$TAG/hbx" > "$O/hbx.txt" 2>&1
    ;;
*)
    echo "unknown part $PART"; exit 2 ;;
esac
