"""Debug: exchange_run step by step on the engine and the oracle; after every
heartbeat compare every node's cache (window 0 holds the recovered copies)."""
import json
import sys

import numpy as np

sys.path[:0] = ["go-libp2p-pubsub_amd", "oracle", "tests"]
import gossip_cases as gc  # noqa: E402
import heartbeat_cases as hc  # noqa: E402
import propagation_cases as pc  # noqa: E402
import gsx  # noqa: E402
import oracle as orc  # noqa: E402
from gsx import abi  # noqa: E402

kw = json.loads(sys.argv[1])
T, n, d, seed = kw.get("T", 2), kw.get("n", 300), kw.get("d", 6), 5
msgs, hops, invalid, ticks = kw.get("msgs", 24), kw.get("hops", 2), kw.get("invalid", 0.0), kw.get("ticks", 8)
bes = [gsx.Engine(T), orc.Oracle(T)]
ov = pc.overlay(n, d, seed)
for be in bes:
    pc.setup(be, ov, T, seed, mesh_degree=6)
    be.set_gossipsub_params(gc.params(max_ihave_length=kw["max_ihave_length"]))
for k in range(ticks):
    now = hc.T0 + (3 + k) * abi.SECOND
    outs = [be.heartbeat(1 + k, now, seed * 31 + 7).as_dict() for be in bes]
    c = [[sorted(be.mcache_ids(v, abi.GSX_ANY_TOPIC, 1).tolist()) for v in range(n)] for be in bes]
    bad = [v for v in range(n) if c[0][v] != c[1][v]]
    print("tick", k, "recovered", outs[0]["gossip_delivered"], outs[1]["gossip_delivered"], "nodes whose window 0 differs", len(bad))
    if bad:
        v = bad[0]
        print("  node", v, "engine-only", sorted(set(c[0][v]) - set(c[1][v]))[:10], "oracle-only", sorted(set(c[1][v]) - set(c[0][v]))[:10])
        break
    for be in bes:
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, max_hops=hops, latency_ms=5, seed=seed + k)
        cfg.now_ns = now + 100 * abi.MILLISECOND
        be.propagate(pc.messages(n, msgs, seed + 1000 * k, invalid=invalid), cfg)
        be.refresh(now + 500 * abi.MILLISECOND)
