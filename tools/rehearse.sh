#!/bin/bash
# N=2 rehearsal of bench.py on one GPU (gloo through host memory, every rank on
# device 0): plan exchange, per-hop all-to-all (compacted, then dense in chunks),
# credit all-reduce, the sharded heartbeat with the gossip exchange (cfg5 leg).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run TAG EXTRA...
    local tag=$1
    shift
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --no-cpu --peers 500000 \
        --prop-peers 2000000 --prop-steps 2 --adv-peers 400000 --hb-steps 2 "$@" > gpurun_out/rehearse_$tag.log 2>&1
    local rc=$?
    grep '^{' gpurun_out/rehearse_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['propagation']; a=d['adversarial']; print(json.dumps({'value': d['value'], 'replica': {k: p['replica'][k] for k in ('value','ms_per_batch','deliveries_per_batch')}, 'sharded': {k: p['sharded'][k] for k in ('value','ms_per_batch','deliveries_per_batch','hops','exchange')}, 'cfg5_heartbeat_ms': a.get('heartbeat_ms_rounds'), 'cfg5_forwarding_exchange': a.get('forwarding_exchange'), 'cfg5_heartbeat_first_round': {k: a['heartbeat_first_round'][k] for k in ('iwant_msgs','gossip_delivered','fwd_delivered','grafts','prunes')}}))" || tail -20 gpurun_out/rehearse_$tag.log
    return $rc
}
run compact && run dense --shard-exchange dense --shard-chunk 4
