#!/bin/bash
# One GPU call: the default bench line, a rocprofv3 kernel-trace summary of the
# same bench, then the PMC byte passes of tools/pmc_r03.sh.  Each GPU step has
# its own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-measure}
mkdir -p "$O"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "=== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 2 "$O/$name.err"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python3 bench.py
[ "${SKIP_KT:-0}" = 1 ] || step kt 600 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- \
    python3 bench.py --steps 10 --no-cpu --no-dropin
[ "${SKIP_PMC:-0}" = 1 ] || step pmc 1000 ./tools/pmc_r03.sh "${1:-measure}/pmc"
echo "measure done"
