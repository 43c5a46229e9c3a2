#!/bin/bash
# Propagation parity tests + per-hop kernel trace (tools/prop_profile.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-x}
make -s -C go-libp2p-pubsub_amd && make -s -C oracle || exit 3
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_propagation.py tests/test_gpu_heartbeat.py \
    -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pprof_$TAG -o kt --output-format csv -- \
    python3 tools/prop_profile.py > gpurun_out/pprof_$TAG.log 2>&1 || exit $?
grep '^{' gpurun_out/pprof_$TAG.log | tail -1
exit $rc
