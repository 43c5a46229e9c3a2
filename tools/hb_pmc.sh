#!/bin/bash
# PMC passes (one counter group per run) over the cfg5 attack rounds
# (tools/adv_micro.py --no-spam): per-dispatch counters of the heartbeat
# kernels, summarised with tools/pmc_table.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/hpmc_${1:-r02}
mkdir -p "$OUT"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- \
        python3 tools/adv_micro.py --no-spam > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i ($C) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
for k in k_hb_recv k_hb_maintain k_hb_answer k_hb_scan; do echo "== $k"; python3 tools/pmc_table.py "$OUT" "$k"; done
