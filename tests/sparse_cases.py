"""BASELINE cfg1: TestSparseGossipsub (gossipsub_test.go:43-82) restated for the
synchronous engine, with scoring on.  20 gossipsub peers join one topic,
connect sparsely (sparseConnect = connectSome(hosts, 3), floodsub_test.go:73-87),
two heartbeats build the mesh (handleGraft accepts), then 100 messages are
published one at a time by a random owner, each as its own propagation call,
and every peer must receive every message.  A heartbeat runs after message 50
(the reference's heartbeat ticks while it publishes).  Loaded identically into
any backend (engine or oracle)."""
from __future__ import annotations

import numpy as np

from gsx import abi, synth

S = abi.SECOND
MS = abi.MILLISECOND
T0 = 1_700_000_000 * S
N = 20
N_MSGS = 100
SEED = 4


def overlay():
    ov = synth.connect_some_overlay(N, d=3, seed=SEED)
    return ov


def connected(ov):
    seen = {0}
    todo = [0]
    while todo:
        u = todo.pop()
        for v in ov.col[ov.row_ptr[u]:ov.row_ptr[u + 1]]:
            if int(v) not in seen:
                seen.add(int(v))
                todo.append(int(v))
    return len(seen) == ov.n


def run(be):
    """-> (heartbeat outs, per-message (PropOut dict, hop [n]))."""
    ov = overlay()
    be.set_peer_params(synth.bench_peer_params())
    be.set_topic_params(0, synth.spam_test_topic_params())
    be.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                     accept_px_threshold=0, opportunistic_graft_threshold=0))
    be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    be.set_app_scores(np.zeros(ov.n_pairs))
    be.apply_events(np.array([(abi.EV_ADD_PEER, 0, p, T0, 0) for p in range(ov.n_pairs)], dtype=abi.event_dtype()))
    hbs = [be.heartbeat(1, T0 + S, SEED).as_dict(), be.heartbeat(2, T0 + 2 * S, SEED).as_dict()]
    owners = synth.h(SEED, synth.TAG_SRC, np.arange(N_MSGS), 0) % np.uint64(N)
    res = []
    for i in range(N_MSGS):
        if i == 50:
            hbs.append(be.heartbeat(3, T0 + 3 * S, SEED).as_dict())
        ms = np.zeros(1, dtype=abi.msg_dtype())
        ms["source"] = int(owners[i])
        ms["msg_id"] = i + 1
        now = T0 + 2 * S + (i + 1) * 10 * MS
        cfg = abi.PropConfig(router=abi.GSX_ROUTER_GOSSIPSUB, topic=0, flood_publish=0, max_hops=20,
                             hop_latency_ns=MS, now_ns=now, credit_scores=abi.GSX_CREDIT_NOW, randomsub_size=0,
                             seed=SEED, validation_delay_ns=0)
        out, hop, _ = be.propagate(ms, cfg, want_results=True)
        res.append((out.as_dict(), hop[0].copy()))
    return hbs, res


def check(hbs, res):
    assert hbs[0]["grafts"] > 0 and hbs[0]["mesh_links"] > 0
    for out, hop in res:
        assert (hop != 0xFF).all()  # every subscriber got the message (sub.Next)
        assert out["deliveries"] == N - 1
