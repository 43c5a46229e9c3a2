#!/bin/bash
# PMC passes over the propagation workload (tools/prop_profile.py), one
# counter group per pass (MI355X_MICROARCH.md: <= 8 SQ, <= 4 TCC per pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/ppmc_${1:-r01}
mkdir -p "$OUT"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- \
        python3 tools/prop_profile.py --batches 1 --msgs ${MSGS:-256} > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i ($C) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
