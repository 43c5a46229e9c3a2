#!/bin/bash
# N=2 rehearsal of bench.py on one GPU (gloo through host memory, every rank on
# device 0): plan exchange, per-hop compacted all-to-all, credit all-reduce.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --no-cpu --peers 500000 \
    --prop-peers 2000000 --prop-steps 2 --adv-peers 400000 --hb-steps 2 > gpurun_out/rehearse.log 2>&1
rc=$?
grep '^{' gpurun_out/rehearse.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['propagation']; print(json.dumps({'value': d['value'], 'replica': {k: p['replica'][k] for k in ('value','ms_per_batch','deliveries_per_batch')}, 'sharded': {k: p['sharded'][k] for k in ('value','ms_per_batch','deliveries_per_batch','hops','exchange')}}))" || tail -20 gpurun_out/rehearse.log
exit $rc
