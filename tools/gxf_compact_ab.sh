#!/bin/bash
# A/B of the forwarding pull's eligible-sender list (GSX_GXF_NO_COMPACT=1: every pair of the row):
# heartbeat rounds with the gossip exchange (tools/hb_micro.py --exchange), each variant its own process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for v in base nocompact base; do
    if [ $v = nocompact ]; then export GSX_GXF_NO_COMPACT=1; else unset GSX_GXF_NO_COMPACT; fi
    echo "== $v"
    timeout -k 10 300 python3 tools/hb_micro.py --exchange --rounds 6 2>/dev/null | grep tick || exit 1
done
