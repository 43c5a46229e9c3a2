#!/bin/bash
# HBM bytes per dispatch of the heartbeat / exchange / forwarding kernels, one
# --pmc pass per counter (tools/pmc_disp.py: 2 x FETCH_SIZE + WRITE_SIZE KiB, gfx950):
#   bash tools/pmc_pull.sh hb    tools/hb_micro.py after the bench settle (heavy-forwarding rounds too)
#   bash tools/pmc_pull.sh adv   tools/adv_micro.py (cfg5: spam batch, attack round, second round)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
set -u
export TMPDIR=/tmp
W=${1:-hb}
O=gpurun_out/pmc_$W
mkdir -p $O
if [ "$W" = adv ]; then CMD="python3 tools/adv_micro.py"; else
    CMD="python3 tools/hb_micro.py --exchange --settle 8 --first-tick 59 --rounds 2"; fi
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $O/w/$C -o pmc --output-format csv -- $CMD > $O/$C.log 2>&1 || exit 1
done
for K in k_gxf_pull k_gxf_mark k_gx_ask k_hb_gossip k_gx_node k_hb_recv_grp k_hb_maintain k_refresh_score k_gx_merge \
         k_gx_setprep k_gxf_init k_prop_hop; do
  python3 tools/pmc_disp.py $O w $K 4
done > $O/summary.txt
find $O/w -name "*.csv" -size +30M -delete
