#!/bin/bash
# PMC passes over the forwarding pull kernel only (tools/hb_micro.py --exchange):
# HBM bytes (FETCH_SIZE, WRITE_SIZE: one pass each), L2 hits/misses, and the
# SQ instruction / wait counters; per-dispatch rows in each pass's CSV.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-gxf_pmc}
mkdir -p "$O"
K=${2:-k_gxf_pull_g}
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVE_CYCLES"; do
    i=$((i + 1))
    echo "=== pass $i: $C $(date +%T)"
    timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex "$K" -d "$O/p$i" -o pmc --output-format csv -- \
        python3 tools/hb_micro.py --exchange --rounds 2 > "$O/p$i.log" 2>&1
    rc=$?
    echo "=== pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 5 "$O/p$i.log"; exit $rc; fi
done
