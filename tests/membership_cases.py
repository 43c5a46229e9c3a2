"""Partial topic membership (gs.p.topics as the "in topic"
filter, Join / Leave, fanout for publishers that have not joined,
gossipsub.go:943-1083, 1517-1554), driven identically through any backend."""
from __future__ import annotations

import numpy as np

import heartbeat_cases as hc
import propagation_cases as pc
from gsx import abi

S = abi.SECOND
MS = abi.MILLISECOND


def joined_bits(n, T, seed, p=(0.7, 0.5, 0.8, 0.6)):
    rng = np.random.default_rng(seed + 55)
    bits = np.zeros(n, dtype=np.uint64)
    for t in range(T):
        bits |= (rng.random(n) < p[t % len(p)]).astype(np.uint64) << np.uint64(t)
    return bits


def membership_run(be, n=400, d=6, T=2, seed=9, ticks=8, msgs=16, fanout_ttl_s=3, join_at=4, leave_at=6):
    """Joined subsets per topic; every round: a heartbeat, then a gossipsub
    batch on topic k % T from random sources (some have not joined: they
    publish through their fanout), then a refresh; at round join_at some
    nodes join, at leave_at some leave.  Returns per-tick counters, snapshots,
    membership exports and propagation outcomes."""
    ov = pc.overlay(n, d, seed)
    pc.setup(be, ov, T, seed, mesh_degree=0)
    be.set_subscriptions(joined_bits(n, T, seed))
    from oracle import default_gossipsub_params

    gp = default_gossipsub_params()
    gp.fanout_ttl_ns = fanout_ttl_s * S
    be.set_gossipsub_params(gp)
    rng = np.random.default_rng(seed + 3)
    outs, snaps, mems, props = [], [], [], []
    for k in range(ticks):
        now = hc.T0 + (3 + k) * S
        if k == join_at:
            nodes = rng.choice(n, 30, replace=False).astype(np.uint32)
            topics = rng.integers(0, T, 30).astype(np.uint32)
            outs.append(("join", be.join(nodes, topics, now - 200 * MS, seed + 1).as_dict()))
        if k == leave_at:
            nodes = rng.choice(n, 20, replace=False).astype(np.uint32)
            topics = rng.integers(0, T, 20).astype(np.uint32)
            outs.append(("leave", be.leave(nodes, topics, now - 100 * MS).as_dict()))
        outs.append(("hb", be.heartbeat(1 + k, now, seed * 31 + 7).as_dict()))
        snaps.append(hc.snapshot(be))
        mems.append(be.export_membership())
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, latency_ms=5, seed=seed + k)
        cfg.now_ns = now + 100 * MS
        out, hop, frm = be.propagate(pc.messages(n, msgs, seed + 1000 * k), cfg, want_results=True)
        props.append((out.as_dict() if hasattr(out, "as_dict") else out, hop))
        be.refresh(now + 500 * MS)
    return ov, outs, snaps, mems, props
