#!/usr/bin/env python3
"""Heartbeat microbenchmark for profiling: the bench's cfg3 state (1M peers x
8 topics), a 256-message gossipsub batch before every round, K rounds from a
chosen tick (default: steady rounds after the warm-up and the
opportunistic-graft round).  Prints per-round wall times.

    python tools/hb_micro.py [--rounds K] [--first-tick 61] [--peers N]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from gsx import abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--first-tick", type=int, default=61)
ap.add_argument("--settle", type=int, default=3,
                help="untimed rounds before the timed ones (bench.py: --settle 8 --first-tick 59)")
ap.add_argument("--peers", type=int, default=1_000_000)
ap.add_argument("--topics", type=int, default=8)
ap.add_argument("--msgs", type=int, default=256)
ap.add_argument("--exchange", action="store_true", help="the gossip exchange (D) on, as in bench.py")
ap.add_argument("--verbose", action="store_true", help="more heartbeat counters per round")
a = ap.parse_args()

ov, e = bench.build_engine(a.peers, a.topics, 6, synth.SEED, 0)
e.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                accept_px_threshold=0, opportunistic_graft_threshold=5))
now = bench.T0
if a.exchange:
    from gsx import engine as gsx_engine_mod

    e.set_gossipsub_params(gsx_engine_mod.default_gossipsub_params(gossip_exchange=1))
args = argparse.Namespace(prop_hops=24)
cfg = bench.prop_config(args, a.peers)
tick = a.first_tick - 1 - a.settle
for k in range(a.settle + a.rounds):
    tick += 1
    now += abi.SECOND
    cfg.now_ns = now - abi.SECOND // 2
    e.propagate(bench.prop_messages(a.peers, a.msgs, 5, first=k * a.msgs), cfg)
    e.settle_scores()  # (as bench.py: the batch's deferred re-scores outside the round)
    e.sync()
    b0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)  # (the profiler's clock: tools/hb_api.py windows)
    t0 = time.perf_counter()
    o = e.heartbeat(tick, now, synth.SEED).as_dict()
    e.sync()
    print(f"window {tick} {b0} {time.clock_gettime_ns(time.CLOCK_BOOTTIME)}", flush=True)
    print(f"{'settle ' if k < a.settle else ''}tick {tick}: {(time.perf_counter() - t0) * 1e3:.3f} ms grafts={o['grafts']} prunes={o['prunes']} "
          f"ihave={o['ihave_msgs']} iwant={o['iwant_msgs']} delivered={o['gossip_delivered']}", flush=True)
    if a.verbose:
        print("   ", {k: o[k] for k in ("ihave_ids", "ihave_ignored", "iwant_ids", "iwant_served", "gossip_rejected",
                                      "gossip_duplicates", "fwd_delivered", "fwd_duplicates", "fwd_graylisted",
                                      "broken_promises", "penalties")}, flush=True)
e.close()
