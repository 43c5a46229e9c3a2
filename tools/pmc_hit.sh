#!/bin/bash
# L2 hit rate of the propagation hop kernels (is the hop's
# line traffic HBM or Infinity Cache?): one rocprofv3 --pmc pass of
# TCC_HIT_sum / TCC_MISS_sum / TCC_EA0_RDREQ_sum over tools/prop_profile.py
# (64- and 1024-message batches), summed per kernel by tools/pmc_hit.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-pmchit}
mkdir -p "$O"
for M in 64 1024; do
    timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace -d "$O/p$M" -o pmc \
        --output-format csv -- python3 tools/prop_profile.py --msgs $M --batches 3 --warmup 2 > "$O/p$M.log" 2>&1 || exit $?
    python3 tools/pmc_hit.py "$O/p$M/pmc_counter_collection.csv" "$O/p$M/pmc_kernel_trace.csv" > "$O/p$M.txt"
    cat "$O/p$M.txt"
done
