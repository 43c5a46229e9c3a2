#!/bin/bash
# Drop-in scorer latency (tools/dropin_latency.cpp) at 100 / 1,000 / 10,000 peers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=go-libp2p-pubsub_amd/gsx
g++ -std=c++17 -O2 tools/dropin_latency.cpp -L$L -lgsx -Wl,-rpath,$PWD/$L -o /tmp/dropin_latency || exit 1
for k in 100 1000 10000; do timeout -k 10 120 /tmp/dropin_latency $k 2000 || exit $?; done
