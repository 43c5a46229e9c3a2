#!/bin/bash
# Kernel traces (bash tools/profile.sh TAG): the propagation workload at 64 / 1024 messages
# (tools/prop_kt.sh) and the cfg5 attack heartbeats after the spam batch
# (tools/adv_micro.py, the bench's adversarial leg alone).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-prof}
mkdir -p gpurun_out/$TAG
bash tools/prop_kt.sh ${TAG}pk > gpurun_out/$TAG/prop_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/adv -o kt --output-format csv -- \
    python3 tools/adv_micro.py > gpurun_out/$TAG/adv.log 2>&1 || exit $?
python3 tools/kt_rounds.py gpurun_out/$TAG/adv/kt_kernel_trace.csv 25 k_gxf_pull k_gxf_mark > gpurun_out/$TAG/adv_rounds.txt
grep -v "^W20\|^E20" gpurun_out/$TAG/prop_kt.log | tail -34
head -60 gpurun_out/$TAG/adv_rounds.txt
grep heartbeat_ms gpurun_out/$TAG/adv.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['heartbeat_ms_rounds'], d['spam'])"
