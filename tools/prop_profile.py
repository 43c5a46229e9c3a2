#!/usr/bin/env python3
"""Propagation-only workload for rocprofv3 (kernel trace / PMC passes):
the bench's replica leg — 1M-peer overlay, gossipsub, 256-message batches."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))
import bench  # noqa: E402
from gsx import abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--peers", type=int, default=1_000_000)
ap.add_argument("--msgs", type=int, default=256)
ap.add_argument("--batches", type=int, default=3)
ap.add_argument("--warmup", type=int, default=0,
                help="batches before the measured ones, then one k_prop_hops_export (gsx_prop_results) as the "
                     "marker tools/pmc_bytes.py counts from (the first call's full fwd / pin passes stay out)")
ap.add_argument("--router", type=int, default=abi.GSX_ROUTER_GOSSIPSUB)
ap.add_argument("--track", type=int, default=0, help="keep first-deliverer rows (gsx_prop_set_tracking)")
ap.add_argument("--credit", type=int, default=abi.GSX_CREDIT_NOW)
ap.add_argument("--latency-us", type=int, default=10_000, help="hop latency (P3 window of the params: 10 ms)")
a = ap.parse_args()
th = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                    accept_px_threshold=0, opportunistic_graft_threshold=0)
e = bench.prop_engine(a.peers, 0, a.peers, 6, synth.SEED, 0, th, None)


class A:
    prop_hops = 24


e.set_prop_tracking(bool(a.track))
cfg = bench.prop_config(A, a.peers)
cfg.router = a.router
cfg.credit_scores = a.credit
cfg.hop_latency_ns = a.latency_us * 1000
for b in range(a.warmup + a.batches):
    if a.warmup and b == a.warmup:
        e.prop_results(a.msgs)  # (read-only: the marker dispatch)
    msgs = bench.prop_messages(a.peers, a.msgs, synth.SEED, first=b * a.msgs)
    t0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)  # (the profiler's clock: tools/hb_api.py windows)
    out = e.propagate(msgs, cfg)[0]
    print(f"window {b} {t0} {time.clock_gettime_ns(time.CLOCK_BOOTTIME)}", flush=True)
    d = out.as_dict()
    print(json.dumps({"batch": b, "hop_kernel_ms": out.hop_kernel_ms, "deliveries": d["deliveries"],
                      "hop_deliveries": d["hop_deliveries"], "edge_sends": out.edge_sends,
                      "new_words": out.new_words}), flush=True)
e.close()
