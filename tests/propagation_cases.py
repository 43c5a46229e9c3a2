"""Shared setup for propagation tests: a seeded overlay, scores, a mesh, and
messages, loaded identically into any backend (engine or oracle)."""
from __future__ import annotations

import numpy as np

from gsx import abi, synth

S = abi.SECOND
T0 = 1_700_000_000 * S


def overlay(n, d, seed, mix_protocols=False, direct_frac=0.0):
    ov = synth.connect_some_overlay(n, d=d, seed=seed)
    rng = np.random.default_rng(seed + 100)
    ef = ov.edge_flags.copy()
    if mix_protocols:  # some peers speak floodsub only (feature Mesh off)
        fl_nodes = rng.random(n) < 0.15
        fl_pair = fl_nodes[ov.col]
        ef[fl_pair] = (ef[fl_pair] & np.uint8(0xFF ^ abi.GSX_EDGE_GOSSIPSUB)) | np.uint8(abi.GSX_EDGE_FLOODSUB)
    if direct_frac > 0:
        ef[rng.random(len(ef)) < direct_frac] |= abi.GSX_EDGE_DIRECT
    ov.edge_flags = ef
    return ov


def setup(be, ov, T, seed, mesh_degree=6, disconnect_frac=0.0, score_spread=True):
    """AddPeer every pair, graft a random mesh (each node grafts up to
    mesh_degree of its gossipsub peers on every topic, GRAFTs accepted both
    ways), optionally disconnect some pairs, random app scores so that some
    peers fall under the publish threshold."""
    rng = np.random.default_rng(seed + 1)
    be.set_peer_params(synth.bench_peer_params())
    for t in range(T):
        tp = synth.spam_test_topic_params()
        tp.mesh_message_deliveries_window_ns = 25 * abi.MILLISECOND  # some late duplicates fall outside
        be.set_topic_params(t, tp)
    be.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                     accept_px_threshold=0, opportunistic_graft_threshold=0))
    be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    E = ov.n_pairs
    ev = [(abi.EV_ADD_PEER, 0, p, T0, 0) for p in range(E)]
    obs = ov.pair_observer()
    # mesh: for each node and topic pick up to mesh_degree gossipsub neighbours
    for t in range(T):
        for i in range(ov.n):
            row = np.arange(ov.row_ptr[i], ov.row_ptr[i + 1])
            row = row[(ov.edge_flags[row] & abi.GSX_EDGE_GOSSIPSUB) != 0]
            pick = rng.permutation(row)[:mesh_degree]
            for q in pick:
                ev.append((abi.EV_GRAFT, t, int(q), T0, 0))
    be.apply_events(np.array(ev, dtype=abi.event_dtype()))
    # make the mesh symmetric-ish: the reverse pair accepts the GRAFT
    st = be.export_state()
    rf = st["rec_flags"].reshape(T, E)
    key = {(int(obs[q]), int(ov.col[q])): q for q in range(E)}
    back = []
    for t in range(T):
        for q in np.nonzero(rf[t] & abi.GSX_REC_IN_MESH)[0]:
            r = key.get((int(ov.col[q]), int(obs[q])))
            if r is not None and not (rf[t][r] & abi.GSX_REC_IN_MESH):
                back.append((abi.EV_GRAFT, t, int(r), T0, 0))
    if back:
        be.apply_events(np.array(back, dtype=abi.event_dtype()))
    if score_spread:
        app = np.where(rng.random(E) < 0.08, -500.0, rng.normal(0, 2, E))
    else:
        app = np.zeros(E)
    be.set_app_scores(app)
    if disconnect_frac > 0:
        rm = np.nonzero(rng.random(E) < disconnect_frac)[0]
        be.apply_events(np.array([(abi.EV_REMOVE_PEER, 0, int(q), T0 + S, 0) for q in rm], dtype=abi.event_dtype()))
    be.refresh(T0 + 2 * S)
    return app


def messages(n_nodes, m, seed, invalid=0.0):
    """`invalid`: fraction of messages validation does not accept (REJECT,
    IGNORE, THROTTLE in 3:1:1), drawn from the seed."""
    ms = np.zeros(m, dtype=abi.msg_dtype())
    ms["source"] = (synth.h(seed, synth.TAG_SRC, np.arange(m), 0) % np.uint64(n_nodes)).astype(np.uint32)
    ms["msg_id"] = np.arange(m, dtype=np.uint64) + 1000 * seed
    if invalid > 0:
        rng = np.random.default_rng(seed + 77)
        bad = rng.random(m) < invalid
        kind = rng.choice([abi.GSX_VALIDATION_REJECT] * 3 + [abi.GSX_VALIDATION_IGNORE, abi.GSX_VALIDATION_THROTTLE], m)
        ms["validation"] = np.where(bad, kind, abi.GSX_VALIDATION_ACCEPT).astype(np.uint32)
    return ms


def config(router, topic=0, flood_publish=0, max_hops=40, latency_ms=10, credit=1, size=0, seed=5, delay_ms=0.0):
    return abi.PropConfig(router=router, topic=topic, flood_publish=flood_publish, max_hops=max_hops,
                          hop_latency_ns=latency_ms * abi.MILLISECOND, now_ns=T0 + 3 * S, credit_scores=credit,
                          randomsub_size=size, seed=seed, validation_delay_ns=int(delay_ms * abi.MILLISECOND))


def with_hub(ov, hub: int, k: int, seed: int, flags=None):
    """ov plus undirected links from `hub` to k random other nodes (a node of
    degree > 256: RandomSub's candidate lists and the heartbeat's hub paths)."""
    import dataclasses

    rng = np.random.default_rng(seed)
    obs = ov.pair_observer()
    edges = {(int(u), int(v)): int(f) for u, v, f in zip(obs, ov.col, ov.edge_flags)}
    f0 = int(ov.edge_flags[0]) if flags is None else flags
    for v in rng.choice(np.arange(ov.n)[np.arange(ov.n) != hub], size=k, replace=False):
        edges.setdefault((hub, int(v)), f0)
        edges.setdefault((int(v), hub), f0)
    keys = sorted(edges)
    row_ptr = np.zeros(ov.n + 1, dtype=np.int64)
    for u, _ in keys:
        row_ptr[u + 1] += 1
    return dataclasses.replace(ov, row_ptr=np.cumsum(row_ptr), col=np.array([v for _, v in keys], dtype=np.int32),
                               edge_flags=np.array([edges[kk] for kk in keys], dtype=np.uint8))
