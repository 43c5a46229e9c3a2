#!/bin/bash
# Hop-kernel build variants (gsx/libgsx_<name>.so, GSX_LIB) at 64 and 1024
# messages: per-batch hop-kernel ms of tools/prop_profile.py.  VARIANTS and
# CHECK (a -k filter of GPU propagation tests run against each variant first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/var
for v in ${VARIANTS:-base}; do
  lib=go-libp2p-pubsub_amd/gsx/libgsx_$v.so
  [ "$v" = base ] && lib=go-libp2p-pubsub_amd/gsx/libgsx.so
  if [ -n "${CHECK:-}" ]; then
    GSX_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "$CHECK" \
        > gpurun_out/var/t_$v.log 2>&1 || { echo "$v: tests failed"; tail -20 gpurun_out/var/t_$v.log; exit 1; }
    echo "$v: $(tail -1 gpurun_out/var/t_$v.log)"
  fi
  for m in ${MSGS:-64 1024}; do
    GSX_LIB=$PWD/$lib timeout -k 10 180 python3 tools/prop_profile.py --msgs $m --batches 4 > gpurun_out/var/p_${v}_$m.log 2>&1 || exit $?
    python3 - "$v" "$m" gpurun_out/var/p_${v}_$m.log <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")]
ms = [r["hop_kernel_ms"] for r in rows[1:]]
print(sys.argv[1], sys.argv[2], "hop_kernel_ms", [round(x, 3) for x in ms], "deliv", rows[-1]["deliveries"])
PY
  done
done
