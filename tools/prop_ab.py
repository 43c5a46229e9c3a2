#!/usr/bin/env python3
"""A/B of propagation code paths on one box: the bench's 1M-peer gossipsub
engine, `--batches` timed batches of `--msgs` messages per variant, each
variant in its own process (the engine reads its GSX_* switches once).

    python tools/prop_ab.py [--msgs 64] [--batches 40] VAR=1[,VAR2=1] ...

"base" is the default build; every other argument is a comma-separated list
of environment switches (GSX_NO_SELF_MARK, GSX_NO_FUSE_DUPS, ...).  Prints
one JSON line per variant: ms per batch (wall), hop-kernel ms per batch."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))
    import bench
    from gsx import abi, synth

    th = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                        accept_px_threshold=0, opportunistic_graft_threshold=0)
    e = bench.prop_engine(a.peers, 0, a.peers, 6, synth.SEED, 0, th, None)

    class A:
        prop_hops = 24

    cfg = bench.prop_config(A, a.peers)
    if a.router == "floodsub":
        cfg.router = abi.GSX_ROUTER_FLOODSUB
    for b in range(3):
        e.propagate(bench.prop_messages(a.peers, a.msgs, synth.SEED, first=b * a.msgs), cfg)
    e.sync()
    t0 = time.perf_counter()
    kms = 0.0
    for b in range(a.batches):
        out = e.propagate(bench.prop_messages(a.peers, a.msgs, synth.SEED, first=(3 + b) * a.msgs), cfg)[0]
        kms += out.hop_kernel_ms
    e.settle_scores()
    e.sync()
    el = time.perf_counter() - t0
    print(json.dumps({"variant": a.variant, "msgs": a.msgs, "router": a.router, "ms_per_batch": el / a.batches * 1e3,
                      "hop_kernel_ms": kms / a.batches, "deliveries": out.as_dict()["deliveries"]}), flush=True)
    e.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=1_000_000)
    ap.add_argument("--msgs", type=int, default=64)
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--router", default="gossipsub")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--variant", default="base")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a)
    for v in ["base"] + a.variants:
        env = dict(os.environ)
        if v != "base":
            for kv in v.split(","):
                k, _, val = kv.partition("=")
                env[k] = val or "1"
        r = subprocess.run([sys.executable, "-u", __file__, "--child", "--variant", v, "--peers", str(a.peers),
                            "--msgs", str(a.msgs), "--batches", str(a.batches), "--router", a.router],
                           env=env, timeout=300)
        if r.returncode != 0:
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
