#!/bin/bash
# Round 5: the shard exchange tests (truncated lists, pending refusals) and the
# N=2 rehearsal of bench.py on one GPU.  Each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_shard.py \
    -k "exchange" > gpurun_out/r05/shard_tests.log 2>&1 || { tail -30 gpurun_out/r05/shard_tests.log; exit 1; }
tail -3 gpurun_out/r05/shard_tests.log
timeout -k 10 700 python -u -m pytest -x -v --timeout 650 --timeout-method thread tests/test_gpu_configs.py \
    -k "sharded_gossip" > gpurun_out/r05/cfg3_shard.log 2>&1 || { tail -30 gpurun_out/r05/cfg3_shard.log; exit 1; }
tail -3 gpurun_out/r05/cfg3_shard.log
