#!/bin/bash
# HBM bytes from rocprofv3 PMC counters (bash tools/pmc.sh TAG; copy the
# summary to profiles/pmc_<round>.json and point bench.py PMC_FILE at it) (one counter per pass, MI355X_MICROARCH.md
# HBM section: FETCH_SIZE x 2 + WRITE_SIZE on gfx950, checked by the calibration
# kernels) for the bench's kernels on the current tree:
#   head  the headline k_refresh_score<8, true> (bench.py, scoring legs only)
#   p1024 / p64  the propagation replica workload (tools/prop_profile.py: 3 batches after 2 warm-up ones)
#   hb    cfg3 heartbeat rounds with the gossip exchange (bench.py's heartbeat leg: its last round)
# then tools/pmc_bytes.py writes the per-launch / per-batch / per-round bytes, each
# section tagged with the workload it measured (bench.py attaches a section's
# bytes only to a leg that ran the same workload).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}
mkdir -p "$O"
run() {  # run NAME SECONDS COUNTER CMD...
    local name=$1 secs=$2 c=$3
    shift 3
    echo "=== $name $c $(date +%T)"
    timeout -s KILL "$secs" rocprofv3 --pmc "$c" --kernel-trace -d "$O/$name/$c" -o pmc --output-format csv -- "$@" \
        > "$O/${name}_$c.log" 2>&1
    local rc=$?
    echo "=== $name $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 5 "$O/${name}_$c.log"; exit $rc; fi
}
# PMC_SECTIONS="calib hb": only those runs (tools/pmc_bytes.py then merges them
# into the summary named by PMC_MERGE, e.g. profiles/pmc_r05.json)
want() { [ -z "${PMC_SECTIONS:-}" ] || [[ " $PMC_SECTIONS " == *" $1 "* ]]; }
for C in FETCH_SIZE WRITE_SIZE; do
    want calib && run calib 120 $C ./tools/microbench/pmc_calib
    want head && run head 300 $C python3 bench.py --steps 5 --warmup 1 --no-cpu --no-dropin --no-single-observer --prop-msgs 0 \
        --prop-peers 0 --hb-steps 0 --adv-peers 0
    want p1024 && run p1024 200 $C python3 tools/prop_profile.py --msgs 1024 --batches 3 --warmup 2
    want p64 && run p64 200 $C python3 tools/prop_profile.py --msgs 64 --batches 3 --warmup 2
    want hb && run hb 300 $C python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin --no-single-observer --prop-msgs 0 \
        --prop-peers 0 --adv-peers 0 --hb-steps 5
done
python3 tools/pmc_bytes.py "$O" "n=1000000,T=8,d=6,E=11999954" ${PMC_MERGE:-} > "$O/summary.json" && cat "$O/summary.json"
