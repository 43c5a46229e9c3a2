#!/usr/bin/env python3
"""cfg5 adversarial leg of bench.py alone (4M peers, 20 % sybils, spam batch,
two heartbeats), for profiling:

    python tools/adv_micro.py [--peers N] [--no-spam]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--peers", type=int, default=4_000_000)
ap.add_argument("--no-spam", action="store_true")
a = ap.parse_args()
args = argparse.Namespace(adv_peers=a.peers, steps=2, prop_msgs=0 if a.no_spam else 1024, prop_hops=24,
                          rehearse=False, hb_steps=1)
out = bench.adversarial_leg(args, 0, 1, 0, None, "cuda:0")
print(json.dumps(out), flush=True)
