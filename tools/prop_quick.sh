#!/bin/bash
# Propagation-only GPU check: parity tests of the propagation path, then the
# 1M replica leg under a kernel trace (per-kernel averages in
# gpurun_out/pq/kt_kernel_stats.csv).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C go-libp2p-pubsub_amd && make -s -C oracle || exit 3
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "${TESTS:-prop or smoke or shard}" \
    > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pq -o kt --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu --prop-peers 0 --adv-peers 0 --hb-steps 0 --prop-steps 10 \
    > gpurun_out/b.log 2>&1
rc=$?
grep -o '"replica": {[^}]*}' gpurun_out/b.log
head -16 gpurun_out/pq/kt_kernel_stats.csv | cut -d, -f1-4
exit $rc
