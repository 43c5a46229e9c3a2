#!/bin/bash
# HBM bytes per dispatch of the forwarding pulls and the heartbeat exchange kernels
# (tools/hb_micro.py with the bench settle: its heavy-forwarding rounds), one --pmc pass per counter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
set -u
export TMPDIR=/tmp
O=gpurun_out/pmcpull
mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d $O/hb/$C -o pmc --output-format csv -- python3 tools/hb_micro.py --exchange --settle 8 --first-tick 59 --rounds 2 > $O/hb_$C.log 2>&1 || exit 1
done
python3 tools/pmc_disp.py $O hb k_gxf_pull 14 > $O/pull.txt
python3 tools/pmc_disp.py $O hb k_gxf_mark 4 >> $O/pull.txt
python3 tools/pmc_disp.py $O hb k_gx_ask 4 >> $O/pull.txt
python3 tools/pmc_disp.py $O hb k_hb_gossip 4 >> $O/pull.txt
python3 tools/pmc_disp.py $O hb k_gx_node 4 >> $O/pull.txt
find $O/hb -name "*.csv" -size +30M -delete
