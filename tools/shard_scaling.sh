#!/bin/bash
# Range-sharded cfg4 (10M peers, 64-message gossipsub batches) in 1, 2, 4, 8
# shards on one GPU (tools/shard_scaling.py), the replicated-frontier exchange
# and the per-pair one, plus a rocprofv3 kernel trace of the 8-shard run.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-shard_scaling}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$R/tools/shard_scaling.py" --shards 2,4,8 > "$OUT/scaling.jsonl" 2> "$OUT/scaling.err" &&
timeout -k 10 600 python3 "$R/tools/shard_scaling.py" --shards 2,8 --no-single --pairs > "$OUT/scaling_pairs.jsonl" 2> "$OUT/scaling_pairs.err" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$R/tools/shard_scaling.py" --shards 8 --batches 3 --no-single > "$OUT/prof_out.jsonl" 2> "$OUT/prof_err.log"
