#!/usr/bin/env python3
"""Per-call overhead of 64-message gossipsub batches (the bench's replica
engine): ms per batch with the message cache growing (every batch kept, as
in the bench leg: a fresh seen buffer per call) against the cache cleared
before every batch (buffers recycled), and floodsub (no cache) beside."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))
import bench  # noqa: E402
from gsx import abi, synth  # noqa: E402

n = 1_000_000
th = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                    accept_px_threshold=0, opportunistic_graft_threshold=0)
e = bench.prop_engine(n, 0, n, 6, synth.SEED, 0, th, None)


class A:
    prop_hops = 24


cfg = bench.prop_config(A, n)
for label, router, clear in (("gossipsub_grow", abi.GSX_ROUTER_GOSSIPSUB, False),
                             ("gossipsub_clear", abi.GSX_ROUTER_GOSSIPSUB, True),
                             ("floodsub", abi.GSX_ROUTER_FLOODSUB, False)):
    cfg.router = router
    e.propagate(bench.prop_messages(n, 64, 7, first=0), cfg)
    e.sync()
    t_all, k_all = 0.0, 0.0
    for b in range(12):
        if clear:
            e.mcache_clear()
        msgs = bench.prop_messages(n, 64, 7, first=(1 + b) * 64)
        t0 = time.perf_counter()
        out = e.propagate(msgs, cfg)[0]
        t_all += time.perf_counter() - t0
        k_all += out.hop_kernel_ms
    print(f"{label}: {t_all / 12 * 1e3:.3f} ms per batch, hop kernels {k_all / 12:.3f} ms", flush=True)
e.close()
