"""Peer exchange on PRUNE (gossipsub.go:811-843, 861-910, 1814-1850) under the
synchronous-round contract of gsx.h, driven identically through the engine
or the oracle: a hand-built star whose hub prunes its oversized mesh, and a
seeded multi-round mesh run with PX on.
"""
from __future__ import annotations

import numpy as np

import heartbeat_cases as hc
import propagation_cases as pc
from gsx import abi

S = abi.SECOND
T0 = pc.T0


def _px_params(prune_peers=16):
    gp = hc.be_default_params()
    gp.do_px = 1
    gp.prune_peers = prune_peers
    return gp


def star_case(be, n_leaves=14, leaf_view=0.0, hub_view=None, no_px=False, prune_peers=16, accept_px=0.0,
              px_log=1 << 12):
    """Hub 0 with a mesh of n_leaves > Dhi leaves, each leaf connected to the
    hub only.  The hub's heartbeat prunes the mesh down to D; every pruned
    leaf gets a PX list of the hub's other peers with score >= 0 (at most
    PrunePeers) and, if its score of the hub (leaf_view) is >= AcceptPXThreshold,
    records all of them as connection candidates (it is connected to none).
    hub_view: {leaf: the hub's app score of it} (negative: pruned without PX
    and left out of every list).  Returns (out dict, px records, pair map)."""
    n = n_leaves + 1
    edges = {}
    flags = abi.GSX_EDGE_GOSSIPSUB | abi.GSX_EDGE_OUTBOUND
    for k in range(1, n):
        edges[(0, k)] = flags | (abi.GSX_EDGE_NO_PX if no_px else 0)
        edges[(k, 0)] = abi.GSX_EDGE_GOSSIPSUB
    row_ptr, col, ef, ips, pair = hc._csr(n, edges)
    be.set_peer_params(abi.PeerScoreParams(app_specific_weight=1.0, app_specific_score_set=1,
                                           decay_interval_ns=S, decay_to_zero=0.01,
                                           behaviour_penalty_decay=0.5, retain_score_ns=S))
    be.set_topic_params(0, hc._zero_weight_topic())
    be.set_thresholds(abi.Thresholds(gossip_threshold=-10, publish_threshold=-100, graylist_threshold=-10000,
                                     accept_px_threshold=accept_px, opportunistic_graft_threshold=-1))
    be.set_gossipsub_params(_px_params(prune_peers))
    be.hb_set_px_log(px_log)
    be.load_overlay(row_ptr, col, ef, ips)
    E = len(col)
    ev = [(abi.EV_ADD_PEER, 0, p, T0, 0) for p in range(E)]
    ev += [(abi.EV_GRAFT, 0, pair[(0, k)], T0, 0) for k in range(1, n)]
    ev += [(abi.EV_GRAFT, 0, pair[(k, 0)], T0, 0) for k in range(1, n)]
    be.apply_events(np.array(ev, dtype=abi.event_dtype()))
    app = np.zeros(E)
    for k in range(1, n):
        app[pair[(k, 0)]] = leaf_view
    for k, v in (hub_view or {}).items():
        app[pair[(0, k)]] = v
    be.set_app_scores(app)
    be.refresh(T0 + S)
    out = be.heartbeat(1, T0 + 2 * S, 4321)
    return out.as_dict(), be.hb_px_records(), pair


def px_run(be, n, d, T, seed, ticks, mesh_degree=14, no_px_frac=0.1, accept_px=0.0, prune_peers=16,
           direct=0.02, disconnect=0.03, join_frac=1.0, prop_msgs=0, d_hi=12):
    """pc.setup's random mesh (meshes above Dhi: the first round prunes
    many), some pairs without feature PX, partial subscriptions (GRAFTs of
    unjoined topics switch PX off for their RPC), then `ticks` rounds of
    heartbeat [+ propagation] + refresh.  Returns (per-round counters,
    per-round px records, per-round snapshots)."""
    ov = pc.overlay(n, d, seed, mix_protocols=True, direct_frac=direct)
    rng = np.random.default_rng(seed + 77)
    ef = ov.edge_flags.copy()
    ef[rng.random(len(ef)) < no_px_frac] |= abi.GSX_EDGE_NO_PX
    ov.edge_flags = ef
    pc.setup(be, ov, T, seed, mesh_degree=mesh_degree, disconnect_frac=disconnect)
    # 8 % of the pairs at -500 (pruned without PX), the rest mostly >= 0 (listed)
    be.set_app_scores(np.where(rng.random(ov.n_pairs) < 0.08, -500.0, np.abs(rng.normal(1, 2, ov.n_pairs))))
    be.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                     accept_px_threshold=accept_px, opportunistic_graft_threshold=0))
    if join_frac < 1.0:
        joined = np.zeros(n, dtype=np.uint64)
        for t in range(T):
            joined |= (rng.random(n) < join_frac).astype(np.uint64) << np.uint64(t)
        be.set_subscriptions(joined)
    gp = _px_params(prune_peers)
    gp.d_hi = d_hi  # Dhi = D: meshes (A) leaves full reject GRAFTs of inbound peers (answers with PX)
    be.set_gossipsub_params(gp)
    be.hb_set_px_log(1 << 22)
    outs, recs, snaps = [], [], []
    for k in range(ticks):
        now = T0 + (3 + k) * S
        outs.append(be.heartbeat(1 + k, now, seed * 31 + 7).as_dict())
        recs.append(be.hb_px_records())
        snaps.append(hc.snapshot(be))
        if prop_msgs:
            cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, latency_ms=5, seed=seed + k)
            cfg.now_ns = now + 100 * abi.MILLISECOND
            be.propagate(pc.messages(n, prop_msgs, seed + 1000 * k), cfg)
        be.refresh(now + 500 * abi.MILLISECOND)
    return ov, outs, recs, snaps


def px_member_run(be, n=500, d=8, T=2, seed=13):
    """PX in Join / Leave rounds (gsx.h): a mesh with partial subscriptions,
    some nodes leave a topic (every Leave PRUNE carries PX), others join one
    (their GRAFTs' answers may).  Returns per-call (counters, px records)."""
    ov = pc.overlay(n, d, seed, mix_protocols=True, direct_frac=0.02)
    rng = np.random.default_rng(seed + 5)
    pc.setup(be, ov, T, seed, mesh_degree=4, disconnect_frac=0.02)
    be.set_app_scores(np.where(rng.random(ov.n_pairs) < 0.08, -500.0, np.abs(rng.normal(1, 2, ov.n_pairs))))
    joined = np.zeros(n, dtype=np.uint64)
    for t in range(T):
        joined |= (rng.random(n) < 0.8).astype(np.uint64) << np.uint64(t)
    be.set_subscriptions(joined)
    gp = _px_params(prune_peers=5)
    gp.d_hi = 6
    be.set_gossipsub_params(gp)
    be.hb_set_px_log(1 << 20)
    res = []
    now = T0 + 3 * S
    res.append((be.heartbeat(1, now, seed).as_dict(), be.hb_px_records()))
    leavers = np.nonzero((joined & np.uint64(1)) != 0)[0][:40].astype(np.uint32)
    out = be.leave(leavers, np.zeros(len(leavers), dtype=np.uint32), now + S)
    res.append((out.as_dict(), be.hb_px_records()))
    joiners = np.nonzero((joined & np.uint64(2)) == 0)[0][:40].astype(np.uint32)
    out = be.join(joiners, np.ones(len(joiners), dtype=np.uint32) if T > 1 else np.zeros(len(joiners), dtype=np.uint32),
                  now + 2 * S, seed + 1)
    res.append((out.as_dict(), be.hb_px_records()))
    return res
