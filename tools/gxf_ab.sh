#!/bin/bash
# A/B of forwarding-pull variants: tools/hb_micro.py --exchange under a kernel
# trace once per GSX_* environment setting given, e.g.
#   tools/gxf_ab.sh TAG GSX_GXF_B=1 GSX_GXF_B=2 GSX_GXF_B=4
# then per variant the per-round gx kernel totals (tools/hop_dump.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
for V in "$@"; do
    echo "=== $V $(date +%T)"
    env "$V" timeout -k 10 200 rocprofv3 --kernel-trace -d "$O/$V" -o kt --output-format csv -- \
        python3 tools/hb_micro.py --exchange --rounds 4 > "$O/$V.log" 2>&1
    rc=$?
    echo "=== $V rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 5 "$O/$V.log"; exit $rc; fi
    grep tick "$O/$V.log"
    python3 tools/hop_dump.py "$O/$V/kt_kernel_trace.csv"
done
