#!/bin/bash
# One-word hop kernel (k_prop_hop_fast1): lanes-per-node x rounds variants
# (GSX_HOP_GR) against the word-split kernel (GSX_HOP_NO_FAST1), 64-message
# batches of tools/prop_profile.py; TESTS=1 runs the propagation GPU tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/f1
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "prop or shard or smoke or config or spam or adversarial or trace or gossip or member" \
      --timeout 300 --timeout-method thread > gpurun_out/f1/tests.log 2>&1 || { tail -20 gpurun_out/f1/tests.log; exit 1; }
  tail -1 gpurun_out/f1/tests.log
fi
for v in ${VARIANTS:-old 42 41 81 82 22}; do
  if [ "$v" = old ]; then e="GSX_HOP_NO_FAST1=1"; else e="GSX_HOP_GR=$v"; fi
  env $e timeout -k 10 120 python3 tools/prop_profile.py --msgs 64 --batches 4 > gpurun_out/f1/p_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/f1/p_$v.log <<'PY'
import json, sys
r = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")]
print(sys.argv[1], [round(x["hop_kernel_ms"], 3) for x in r[1:]], r[-1]["deliveries"], r[-1]["edge_sends"])
PY
done
