#!/bin/bash
# A/B of the forwarding pull's launch shape (GSX_GXF_G lanes per receiver,
# GSX_GXF_B, GSX_GXF_GRID) on tools/hb_micro.py's rounds after the bench
# settle (ticks 56, 57, 59, 60 forward recovered messages to most nodes; 61-63 light)
# and tools/adv_micro.py's cfg5 attack round.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out/ab
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 tools/hb_micro.py --exchange --settle 8 --first-tick 59 --rounds 5 > gpurun_out/ab/$tag.txt 2>&1 || { echo "fail $tag"; exit 1; }
  echo "$tag: $(grep -E '^(settle )?tick (56|57|59|60|61|62|63):' gpurun_out/ab/$tag.txt | awk '{for(i=1;i<=NF;i++) if($i=="ms") printf "%s ", $(i-1)}')"
}
adv() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/adv_micro.py > gpurun_out/ab/adv_$tag.txt 2>&1 || { echo "fail adv $tag"; exit 1; }
  echo "adv $tag: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print([round(x, 2) for x in d['heartbeat_ms_rounds']], round(d['spam']['ms_per_batch'], 2))" gpurun_out/ab/adv_$tag.txt)"
}
for spec in "${@:-base:X=1}"; do
  tag=${spec%%:*}; envs=${spec#*:}
  run "$tag" ${envs//,/ }
  adv "$tag" ${envs//,/ }
done
