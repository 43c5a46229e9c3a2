"""Shared heartbeat scenarios, driven identically through any backend (the
engine or the oracle): a seeded mesh run over several heartbeats, and two
hand-built cases restating reference tests in the synchronous-round model.
"""
from __future__ import annotations

import numpy as np

import propagation_cases as pc
from gsx import abi

S = abi.SECOND
MS = abi.MILLISECOND
T0 = pc.T0


def snapshot(be):
    """Everything a heartbeat can change: records, pair state, backoff, scores."""
    st = be.export_state()
    st["backoff"] = be.export_backoff()
    st["scores"] = be.scores()
    st["ihave_len"], st["ihave_digest"] = be.gossip_results()
    return st


def mesh_run(be, n, d, T, seed, ticks, mesh_degree=6, mix=False, direct=0.0, disconnect=0.0, gp=None,
             prop_msgs=0, first_tick=1, mostly_positive=False):
    """pc.setup's random mesh, then `ticks` rounds of: heartbeat, optional
    gossipsub propagation with score credits, refresh.  Returns the per-tick
    counters and snapshots."""
    ov = pc.overlay(n, d, seed, mix_protocols=mix, direct_frac=direct)
    pc.setup(be, ov, T, seed, mesh_degree=mesh_degree, disconnect_frac=disconnect)
    if mostly_positive:  # 8 % of the pairs at -500, the rest >= 0: meshes can fill up
        rng = np.random.default_rng(seed + 2)
        E = ov.n_pairs
        be.set_app_scores(np.where(rng.random(E) < 0.08, -500.0, np.abs(rng.normal(0, 2, E))))
    if gp is not None:
        be.set_gossipsub_params(gp)
    outs, snaps = [], []
    for k in range(ticks):
        tick = first_tick + k
        now = T0 + (3 + k) * S
        outs.append(be.heartbeat(tick, now, seed * 31 + 7).as_dict())
        snaps.append(snapshot(be))
        if prop_msgs:
            cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, latency_ms=5, seed=seed + k)
            cfg.now_ns = now + 100 * MS
            be.propagate(pc.messages(n, prop_msgs, seed + 1000 * k), cfg)
        be.refresh(now + 500 * MS)
    return ov, outs, snaps


def _csr(n, edges):
    """edges: {(u, v): flags} for the pair u -> v -> (row_ptr, col, flags, ips)."""
    keys = sorted(edges)
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    for u, _ in keys:
        row_ptr[u + 1] += 1
    row_ptr = np.cumsum(row_ptr)
    col = np.array([v for _, v in keys], dtype=np.int32)
    ef = np.array([edges[k] for k in keys], dtype=np.uint8)
    ips = np.full((n, 2), abi.GSX_NO_IP, dtype=np.uint32)
    ips[:, 0] = np.arange(n, dtype=np.uint32)
    return row_ptr, col, ef, ips, {k: i for i, k in enumerate(keys)}


def _zero_weight_topic():
    # the scorer must track inMesh for the topic, but contribute nothing
    return abi.TopicScoreParams(topic_weight=0.0, time_in_mesh_quantum_ns=S, first_message_deliveries_decay=0.5,
                                mesh_message_deliveries_decay=0.5, mesh_failure_penalty_decay=0.5,
                                invalid_message_deliveries_decay=0.5, mesh_message_deliveries_window_ns=MS,
                                mesh_message_deliveries_activation_ns=S)


def opportunistic_graft_case(be):
    """TestGossipsubOpportunisticGrafting (gossipsub_test.go:1663-1811) in
    miniature: node 0 has a mesh of six peers scoring 0, below the
    opportunistic graft threshold 1, and four non-mesh peers scoring 5.  On an
    OpportunisticGraftTicks tick it grafts exactly OpportunisticGraftPeers = 2
    of the better peers, which accept.  Peers 1..10 see node 0 without the
    mesh feature, so they never graft it themselves.  Returns (out, pair map)."""
    n = 11
    edges = {}
    for k in range(1, n):
        edges[(0, k)] = abi.GSX_EDGE_GOSSIPSUB | abi.GSX_EDGE_OUTBOUND
        edges[(k, 0)] = 0
    row_ptr, col, ef, ips, pair = _csr(n, edges)
    be.set_peer_params(abi.PeerScoreParams(app_specific_weight=1.0, app_specific_score_set=1,
                                           decay_interval_ns=S, decay_to_zero=0.01,
                                           behaviour_penalty_decay=0.5, retain_score_ns=S))
    be.set_topic_params(0, _zero_weight_topic())
    be.set_thresholds(abi.Thresholds(gossip_threshold=-10, publish_threshold=-100, graylist_threshold=-10000,
                                     opportunistic_graft_threshold=1))
    be.load_overlay(row_ptr, col, ef, ips)
    E = len(col)
    ev = [(abi.EV_ADD_PEER, 0, p, T0, 0) for p in range(E)]
    ev += [(abi.EV_GRAFT, 0, pair[(0, k)], T0, 0) for k in range(1, 7)]
    ev += [(abi.EV_GRAFT, 0, pair[(k, 0)], T0, 0) for k in range(1, 7)]
    be.apply_events(np.array(ev, dtype=abi.event_dtype()))
    app = np.zeros(E)
    for k in range(7, 11):
        app[pair[(0, k)]] = 5.0
    be.set_app_scores(app)
    be.refresh(T0 + S)
    out = be.heartbeat(60, T0 + 2 * S, 1234)
    return out, pair


def graft_flood_case(be):
    """TestGossipsubAttackGRAFTDuringBackoff (gossipsub_spam_test.go:365-613)
    as heartbeat rounds: node 0 (legit) has the attacker (node 1) backed off
    after a PRUNE; the attacker ignores its own backoff (the test clears it
    before each round) and GRAFTs every round.  Rounds 20 ms apart with
    PruneBackoff 200 ms and GraftFloodThreshold 100 ms: the first GRAFT lands
    after the flood cutoff (one P7 penalty), the next ones before it (two).
    Returns the per-round (out, legit's score of the attacker, backoff)."""
    n = 2
    edges = {(0, 1): abi.GSX_EDGE_GOSSIPSUB, (1, 0): abi.GSX_EDGE_GOSSIPSUB | abi.GSX_EDGE_OUTBOUND}
    row_ptr, col, ef, ips, pair = _csr(n, edges)
    be.set_peer_params(abi.PeerScoreParams(app_specific_score_set=1, behaviour_penalty_weight=-100,
                                           behaviour_penalty_decay=0.01 ** (1 / 60), decay_interval_ns=S,
                                           decay_to_zero=0.01, retain_score_ns=S))
    be.set_topic_params(0, _zero_weight_topic())
    be.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-500, graylist_threshold=-1000))
    gp = be_default_params()
    gp.prune_backoff_ns = 200 * MS
    gp.graft_flood_threshold_ns = 100 * MS
    be.set_gossipsub_params(gp)
    be.load_overlay(row_ptr, col, ef, ips)
    be.apply_events(np.array([(abi.EV_ADD_PEER, 0, p, T0, 0) for p in range(2)], dtype=abi.event_dtype()))
    a_to_l, l_to_a = pair[(1, 0)], pair[(0, 1)]
    # the legit host pruned the attacker 101 ms before the first round
    t1 = T0 + S
    b = np.zeros((1, 2), dtype=np.int64)
    b[0, l_to_a] = t1 - 101 * MS + 200 * MS
    be.import_backoff(b)
    rounds = []
    for k in range(4):
        now = t1 + k * 20 * MS if k < 3 else t1 + 2 * 20 * MS + 201 * MS
        b = be.export_backoff()
        b[0, a_to_l] = 0  # the attacker ignores its backoff
        be.import_backoff(b)
        out = be.heartbeat(k + 1, now, 99)
        rounds.append((out.as_dict(), float(be.scores()[l_to_a]), be.export_backoff().copy()))
    return rounds, pair


def be_default_params():
    import oracle as orc

    return orc.default_gossipsub_params()


def message_cache_case(be):
    """TestMessageCache (mcache_test.go:11-154) through the engine: a cache
    with HistoryGossip 3 / HistoryLength 5; node 0 publishes 10 messages per
    window (one gossipsub batch, ids 0..59 in order), heartbeats Shift the
    windows.  Returns the GetGossipIDs / whole-cache views the test checks."""
    n = 2
    edges = {(0, 1): abi.GSX_EDGE_GOSSIPSUB, (1, 0): abi.GSX_EDGE_GOSSIPSUB}
    row_ptr, col, ef, ips, _ = _csr(n, edges)
    be.set_peer_params(abi.PeerScoreParams(app_specific_score_set=1, decay_interval_ns=S, decay_to_zero=0.01,
                                           behaviour_penalty_decay=0.5, retain_score_ns=S))
    be.set_topic_params(0, _zero_weight_topic())
    be.set_thresholds(abi.Thresholds(gossip_threshold=-10, publish_threshold=-100, graylist_threshold=-1000))
    gp = be_default_params()
    gp.history_gossip, gp.history_length = 3, 5
    be.set_gossipsub_params(gp)
    be.load_overlay(row_ptr, col, ef, ips)
    be.apply_events(np.array([(abi.EV_ADD_PEER, 0, p, T0, 0) for p in range(2)], dtype=abi.event_dtype()))
    views = {}

    def put(lo, hi):
        ms = np.zeros(hi - lo, dtype=abi.msg_dtype())
        ms["source"] = 0
        ms["msg_id"] = np.arange(lo, hi, dtype=np.uint64)
        be.propagate(ms, pc.config(abi.GSX_ROUTER_GOSSIPSUB, max_hops=2, credit=0))

    tick = [0]

    def shift():
        tick[0] += 1
        be.heartbeat(tick[0], T0 + tick[0] * S, 3)

    put(0, 10)
    views["first"] = be.mcache_ids(0, 0, 3)
    shift()
    put(10, 20)
    views["second"] = be.mcache_ids(0, 0, 3)
    views["second_all"] = be.mcache_ids(0, abi.GSX_ANY_TOPIC, 5)
    for lo in (20, 30, 40, 50):
        shift()
        put(lo, lo + 10)
    views["cache"] = be.mcache_ids(0, abi.GSX_ANY_TOPIC, 5)
    views["gossip"] = be.mcache_ids(0, 0, 3)
    views["receiver"] = be.mcache_ids(1, 0, 3)  # node 1 Put what it received too
    return views
