"""Propagation on the GPU (through the C ABI) vs the CPU oracle: delivery sets,
arrival hops, first deliverers, counters and the P2/P3 credits, bit-exact."""
import numpy as np
import pytest

import gsx
import oracle as orc
import propagation_cases as pc
from gsx import abi, synth

pytestmark = pytest.mark.gpu

CASES = [
    # n, d, T, router, flood_publish, m, latency_ms, mix, direct, disconnect
    (300, 3, 1, abi.GSX_ROUTER_FLOODSUB, 0, 64, 10, False, 0.0, 0.0),
    (500, 6, 2, abi.GSX_ROUTER_GOSSIPSUB, 0, 100, 10, True, 0.05, 0.05),
    (500, 6, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 130, 10, True, 0.02, 0.0),
    (800, 4, 1, abi.GSX_ROUTER_RANDOMSUB, 0, 64, 10, True, 0.0, 0.03),
    (2000, 8, 1, abi.GSX_ROUTER_RANDOMSUB, 0, 70, 1, False, 0.0, 0.0),
    (3000, 6, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 192, 1, False, 0.0, 0.0),
    # one-word calls (k_prop_hop_fast1 in the "late" mode: senders split over 4 lanes)
    (1500, 7, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 50, 10, True, 0.03, 0.02),
    (1200, 9, 2, abi.GSX_ROUTER_GOSSIPSUB, 1, 64, 1, False, 0.0, 0.03),
    (900, 14, 1, abi.GSX_ROUTER_FLOODSUB, 0, 33, 10, True, 0.02, 0.0),
    # wide batches: the hop kernel's lane groups (2 lanes per node at 8 words,
    # 4 at 16 and 32 words) and the one-lane multi-chunk walk (12 words)
    (600, 4, 1, abi.GSX_ROUTER_RANDOMSUB, 0, 480, 10, True, 0.0, 0.03),
    (600, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 520, 1, True, 0.02, 0.02),
    (700, 6, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 1000, 10, True, 0.02, 0.0),
    (900, 6, 2, abi.GSX_ROUTER_GOSSIPSUB, 0, 1024, 1, False, 0.0, 0.05),
    (500, 6, 2, abi.GSX_ROUTER_FLOODSUB, 0, 2000, 1, False, 0.0, 0.0),
]


@pytest.mark.parametrize("track", [True, False, "late"], ids=["rows", "counts", "counts-late"])
@pytest.mark.parametrize("case", CASES, ids=[f"r{c[3]}-n{c[0]}-m{c[5]}" for c in CASES])
def test_propagation_matches_oracle(gpu_ok, case, track):
    """track=False: no first-deliverer rows (gsx_prop_set_tracking), the
    duplicate accounting counts the `from` exclusion instead of masking it;
    every counter, hop, credit and score must still match.  "late": the same
    with zero hop latency, so every duplicate is inside the P3 window and the
    hops only move first receipts (the lean hop kernel for flood/gossipsub)."""
    n, d, T, router, fp, m, lat, mix, direct, disc = case
    if track == "late":
        track, lat = False, 0
    seed = n + m
    ov = pc.overlay(n, d, seed, mix_protocols=mix, direct_frac=direct)
    ms = pc.messages(n, m, seed)
    cfg = pc.config(router, topic=T - 1, flood_publish=fp, latency_ms=lat, size=50)
    res = []
    eng = gsx.Engine(T)
    eng.set_prop_tracking(track)
    for be in (eng, orc.Oracle(T)):
        pc.setup(be, ov, T, seed, disconnect_frac=disc)
        out, hop, frm = be.propagate(ms, cfg, want_results=True)
        res.append((out.as_dict(), hop, frm, be.export_state(), be.scores()))
    (go, gh, gf, gs, gsc), (wo, wh, wf, ws, wsc) = res
    assert go == wo
    assert np.array_equal(gh, wh), np.argwhere(gh != wh)[:5]
    if track:
        assert np.array_equal(gf, wf), np.argwhere(gf != wf)[:5]
    else:
        assert gf is None
    for f in abi.STATE_FIELDS:
        assert np.array_equal(gs[f].view(np.uint8), ws[f].view(np.uint8)), f
    assert np.array_equal(gsc.view(np.uint64), wsc.view(np.uint64))
    assert go["deliveries"] > 0
    if router == abi.GSX_ROUTER_GOSSIPSUB:
        assert go["graylisted"] > 0  # the setup puts ~8 % of the senders below GraylistThreshold
    else:
        assert go["graylisted"] == 0  # floodsub / randomsub: AcceptFrom accepts all


def test_propagation_full_size_properties(gpu_ok):
    """cfg2-style at 100k peers: every message reaches each vertex at most once;
    floodsub arrival hops are BFS distances (checked on a sample of messages
    with a numpy BFS); totals add up."""
    n = 100_000
    ov = pc.overlay(n, 6, seed=9)
    e = gsx.Engine(1)
    e.set_peer_params(synth.bench_peer_params())
    e.set_topic_params(0, synth.spam_test_topic_params())
    e.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    e.synthesize_state(abi.SynthSpec(seed=9, now_ns=pc.T0, fmd_max=10, mmd_max=10, mfp_max=1, imd_max_sybil=0,
                                     p_in_mesh=0.5, graft_window_ns=abi.HOUR, bp_max=0, p_disconnected=0,
                                     p_absent=0, expire_jitter_ns=0, sybil_first_node=n))
    ms = pc.messages(n, 64, seed=9)
    out, hop, frm = e.propagate(ms, pc.config(abi.GSX_ROUTER_FLOODSUB, credit=0), want_results=True)
    assert out.deliveries == int((hop != 0xFF).sum()) - len(ms)
    assert out.transmissions == out.deliveries + out.duplicates
    import scipy.sparse as sp
    from scipy.sparse.csgraph import shortest_path

    A = sp.csr_matrix((np.ones(ov.n_pairs), ov.col, ov.row_ptr), shape=(n, n))
    dist = shortest_path(A, unweighted=True, indices=ms["source"][:4].astype(np.int64))
    for k in range(4):
        reach = np.isfinite(dist[k])
        assert np.array_equal(hop[k][reach].astype(np.int64), dist[k][reach].astype(np.int64))


VCASES = [
    # n, d, T, router, flood_publish, m, latency_ms, delay_ms, invalid, mix
    (700, 6, 2, abi.GSX_ROUTER_GOSSIPSUB, 0, 200, 5, 7.0, 0.25, True),
    (600, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 1024, 10, 3.0, 0.2, True),
    (500, 4, 1, abi.GSX_ROUTER_FLOODSUB, 0, 130, 4, 12.0, 0.3, False),
    (800, 5, 1, abi.GSX_ROUTER_RANDOMSUB, 0, 100, 6, 2.0, 0.2, True),
    (1500, 8, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 60, 5, 1.0, 0.25, True),  # one word: fast1 with drops
]


@pytest.mark.parametrize("track", [True, False, "late"], ids=["rows", "counts", "counts-late"])
@pytest.mark.parametrize("case", VCASES, ids=[f"r{c[3]}-n{c[0]}-m{c[5]}-v{c[7]}" for c in VCASES])
def test_propagation_validation_matches_oracle(gpu_ok, case, track):
    """Validation outcomes (REJECT / IGNORE / THROTTLE: seen, not delivered,
    not forwarded; REJECT adds P4 to the sender) and a validation delay that
    stretches every hop and the P3 window (validation.go:230-351,
    score.go:721-820): counters, hops, first deliverers, P2/P3/P4, scores."""
    n, d, T, router, fp, m, lat, delay, invalid, mix = case
    seed = 3 * n + m
    if track == "late":
        track, lat = False, 0
    ov = pc.overlay(n, d, seed, mix_protocols=mix, direct_frac=0.02)
    ms = pc.messages(n, m, seed, invalid=invalid)
    cfg = pc.config(router, topic=T - 1, flood_publish=fp, latency_ms=lat, size=50, delay_ms=delay)
    res = []
    eng = gsx.Engine(T)
    eng.set_prop_tracking(track)
    for be in (eng, orc.Oracle(T)):
        pc.setup(be, ov, T, seed, disconnect_frac=0.02)
        out, hop, frm = be.propagate(ms, cfg, want_results=True)
        res.append((out.as_dict(), hop, frm, be.export_state(), be.scores()))
    (go, gh, gf, gs, gsc), (wo, wh, wf, ws, wsc) = res
    assert go == wo
    assert go["rejected"] > 0 and go["ignored"] > 0
    assert np.array_equal(gh, wh), np.argwhere(gh != wh)[:5]
    if track:
        assert np.array_equal(gf, wf), np.argwhere(gf != wf)[:5]
    for f in abi.STATE_FIELDS:
        assert np.array_equal(gs[f].view(np.uint8), ws[f].view(np.uint8)), f
    assert np.array_equal(gsc.view(np.uint64), wsc.view(np.uint64))


def _overlay_from_edges(n, edges):
    """Symmetric overlay from undirected edges (u, v); the lower id dials."""
    rows = [[] for _ in range(n)]
    for u, v in edges:
        rows[u].append(v)
        rows[v].append(u)
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    col, ef = [], []
    for i in range(n):
        nb = sorted(set(rows[i]))
        row_ptr[i + 1] = row_ptr[i] + len(nb)
        col += nb
        ef += [abi.GSX_EDGE_GOSSIPSUB | (abi.GSX_EDGE_OUTBOUND if i < j else 0) for j in nb]
    ips = np.stack([np.arange(n, dtype=np.uint32) + 1, np.full(n, 0xFFFFFFFF, dtype=np.uint32)], axis=1)
    return synth.Overlay(n=n, row_ptr=row_ptr, col=np.array(col, dtype=np.int32), edge_flags=np.array(ef, dtype=np.uint8),
                         node_ips=ips, sybil=np.zeros(n, dtype=bool))


def _hub_overlay(n, seed):
    """Node 0 peers with everyone (degree n - 1 > 256), the rest form a ring
    with random chords, plus a few isolated nodes at the end."""
    rng = np.random.default_rng(seed)
    core = n - 5
    edges = [(0, i) for i in range(1, core)]
    edges += [(i, i + 1) for i in range(1, core - 1)]
    edges += [tuple(sorted(rng.choice(np.arange(1, core), 2, replace=False))) for _ in range(core)]
    return _overlay_from_edges(n, [e for e in edges if e[0] != e[1]])


EDGE_CASES = [
    # router, m, max_hops, latency_ms, track
    (abi.GSX_ROUTER_GOSSIPSUB, 300, 40, 10, True),
    (abi.GSX_ROUTER_FLOODSUB, 1100, 40, 0, False),   # late accounting, 18 words (LPN 1, 4-word chunks + pad)
    (abi.GSX_ROUTER_GOSSIPSUB, 200, 1, 0, False),    # cut after hop 1: the last hop still delivers
    (abi.GSX_ROUTER_GOSSIPSUB, 200, 2, 0, False),
    (abi.GSX_ROUTER_FLOODSUB, 4096, 3, 0, False),    # 64 words, cut at hop 3
    (abi.GSX_ROUTER_GOSSIPSUB, 0, 40, 10, True),     # empty batch
]


@pytest.mark.parametrize("case", EDGE_CASES, ids=[f"r{c[0]}-m{c[1]}-h{c[2]}-l{c[3]}" for c in EDGE_CASES])
def test_propagation_edge_cases_match_oracle(gpu_ok, case):
    """A hub of degree ~600 (one lane group walks 600 pairs), isolated nodes
    and isolated sources, batches cut short by max_hops (the late accounting's
    last hop still delivers), a 64-word batch, an empty batch."""
    router, m, max_hops, lat, track = case
    n, T = 640, 1
    ov = _hub_overlay(n, seed=m + max_hops)
    ms = pc.messages(n, m, seed=m + 7)
    if m:
        ms["source"][: min(m, 3)] = [n - 1, n - 2, 0][: min(m, 3)]  # two isolated sources and the hub
    cfg = pc.config(router, max_hops=max_hops, latency_ms=lat)
    res = []
    eng = gsx.Engine(T)
    eng.set_prop_tracking(track)
    for be in (eng, orc.Oracle(T)):
        pc.setup(be, ov, T, seed=5, disconnect_frac=0.02)
        out, hop, frm = be.propagate(ms, cfg, want_results=True)
        res.append((out.as_dict(), hop, frm, be.export_state(), be.scores()))
    (go, gh, gf, gs, gsc), (wo, wh, wf, ws, wsc) = res
    assert go == wo
    assert np.array_equal(gh, wh), np.argwhere(gh != wh)[:5]
    if track:
        assert np.array_equal(gf, wf), np.argwhere(gf != wf)[:5]
    for f in abi.STATE_FIELDS:
        assert np.array_equal(gs[f].view(np.uint8), ws[f].view(np.uint8)), f
    assert np.array_equal(gsc.view(np.uint64), wsc.view(np.uint64))
    if m == 0:
        assert go["deliveries"] == 0 and go["transmissions"] == 0


def test_randomsub_full_hub_matches_oracle(gpu_ok):
    """A node linked to every other node (399 peers): RandomSub's candidate
    lists have no degree cap (they are staged over the node's own pairs)."""
    ov = _hub_overlay(400, seed=1)
    ms = pc.messages(400, 10, seed=3)
    res = []
    for be in (gsx.Engine(1), orc.Oracle(1)):
        pc.setup(be, ov, 1, seed=5)
        out, hop, _ = be.propagate(ms, pc.config(abi.GSX_ROUTER_RANDOMSUB, size=50), want_results=True)
        res.append((out.as_dict(), hop, be.scores()))
    assert res[0][0] == res[1][0] and np.array_equal(res[0][1], res[1][1])
    assert np.array_equal(res[0][2].view(np.uint64), res[1][2].view(np.uint64))


@pytest.mark.parametrize("mix,scores_each", [(False, True), (True, True), (False, False), (True, False),
                                             (False, None), (True, None)],
                         ids=["gossipsub-only", "with-floodsub-peers", "gossipsub-only-lazy", "with-floodsub-peers-lazy",
                              "gossipsub-only-deferred", "with-floodsub-peers-deferred"])
def test_propagation_sequence_reuses_forwarding_state(gpu_ok, mix, scores_each):
    """One engine, many calls: the forwarding state (k_prop_fwd / k_prop_pin)
    is kept between calls while nothing it reads changed and rebuilt after
    GRAFT / PRUNE / RemovePeer events, a refresh, new thresholds, app scores
    (floodsub peers are score-gated), a heartbeat, a topic or router switch.
    Every call must match the oracle running the same sequence.  Without
    scores_each the scores are read only at the end, so the lazy folds'
    stale pairs (PropState::stale) carry across calls, events, raised
    thresholds and heartbeats (which settle them).  With scores_each None
    neither the state nor the scores are read between calls, so the deferred
    folds' sums (PropState::acc_s / acc_f) carry across calls until an event,
    a refresh, new thresholds, a heartbeat or a topic switch folds them."""
    n, T = 600, 2
    ov = pc.overlay(n, 5, seed=31, mix_protocols=mix)
    E = ov.n_pairs
    rng = np.random.default_rng(31)
    eng, ref = gsx.Engine(T), orc.Oracle(T)
    gp = orc.default_gossipsub_params()
    for be in (eng, ref):
        pc.setup(be, ov, T, 31, disconnect_frac=0.02)
    steps = [
        ("gossipsub", None),
        ("gossipsub again", None),
        ("graft+prune", [(abi.EV_GRAFT, 0, int(q), pc.T0 + 3 * pc.S, 0) for q in rng.choice(E, 40, replace=False)]
         + [(abi.EV_PRUNE, 0, int(q), pc.T0 + 3 * pc.S, 0) for q in rng.choice(E, 40, replace=False)]),
        ("remove peers", [(abi.EV_REMOVE_PEER, 0, int(q), pc.T0 + 3 * pc.S, 0) for q in rng.choice(E, 25, replace=False)]),
        ("refresh", "refresh"),
        ("thresholds", "thresholds"),
        ("gossipsub after thresholds", None),
        ("thresholds up", "thresholds up"),  # above the stale pairs' bound: they settle first
        ("app scores", "app"),
        ("heartbeat", "heartbeat"),
        ("topic 1", None),
        ("topic 0 after topic 1", None),  # the fold's topic-term cache: topic 1's cached term, topic 0's recomputed
        ("topic 1 after topic 0", None),
        ("trace deliver", "trace"),  # a record of topic 1 changed outside the fold: every cached term is stale
        ("topic 0 after trace", None),
        ("topic 1 after trace", None),  # (the cache is armed by consecutive folds: a new epoch here)
        ("topic 0 after trace, cached", None),
        ("topic weight", "tparams"),  # topic 1's weight changed: its cached terms are stale
        ("topic 0 after weight", None),
        ("topic 1 after weight", None),
        ("topic 0 after weight, cached", None),
        ("floodsub", None),
        ("gossipsub after floodsub", None),
    ]
    for k, (name, action) in enumerate(steps):
        for be in (eng, ref):
            if isinstance(action, list):
                be.apply_events(np.array(action, dtype=abi.event_dtype()))
            elif action == "refresh":
                be.refresh(pc.T0 + 4 * pc.S)
            elif action == "thresholds":
                be.set_thresholds(abi.Thresholds(gossip_threshold=-50, publish_threshold=-60, graylist_threshold=-300,
                                                 accept_px_threshold=0, opportunistic_graft_threshold=0))
            elif action == "thresholds up":
                be.set_thresholds(abi.Thresholds(gossip_threshold=-0.5, publish_threshold=-1, graylist_threshold=-2,
                                                 accept_px_threshold=0, opportunistic_graft_threshold=0))
            elif action == "app":
                be.set_app_scores(np.where(np.arange(E) % 7 == 0, -1000.0, 1.0))
            elif action == "heartbeat":
                be.set_gossipsub_params(gp)
                be.heartbeat(1, pc.T0 + 5 * pc.S, 77)
            elif action == "trace":
                for q in range(0, E, max(E // 40, 1)):
                    be.trace_deliver(int(q), 10_000 + int(q), 1, pc.T0 + 5 * pc.S)
            elif action == "tparams":
                tp = synth.spam_test_topic_params()
                tp.topic_weight = 0.5
                be.set_topic_params(1, tp)
        router = abi.GSX_ROUTER_FLOODSUB if name == "floodsub" else abi.GSX_ROUTER_GOSSIPSUB
        topic = 1 if name.startswith("topic 1") else 0
        ms = pc.messages(n, 96, seed=100 + k)
        cfg = pc.config(router, topic=topic, latency_ms=10)
        res = [be.propagate(ms, cfg, want_results=True) for be in (eng, ref)]
        (go, gh, _), (wo, wh, _) = res
        assert go.as_dict() == wo.as_dict(), name
        assert np.array_equal(gh, wh), name
        if scores_each is None:
            continue
        gs, ws = eng.export_state(), ref.export_state()
        for f in abi.STATE_FIELDS:
            assert np.array_equal(gs[f].view(np.uint8), ws[f].view(np.uint8)), (name, f)
        if scores_each:
            assert np.array_equal(eng.scores().view(np.uint64), ref.scores().view(np.uint64)), name
    assert np.array_equal(eng.scores().view(np.uint64), ref.scores().view(np.uint64))
    gs, ws = eng.export_state(), ref.export_state()
    for f in abi.STATE_FIELDS:
        assert np.array_equal(gs[f].view(np.uint8), ws[f].view(np.uint8)), f


@pytest.mark.parametrize("flood_publish,scores_each", [(0, True), (1, True), (0, False), (1, False)])
def test_credit_threshold_crossings_between_calls(gpu_ok, flood_publish, scores_each):
    """Consecutive gossipsub calls whose own credits move scores across the
    graylist and publish thresholds (invalid messages: P4): the fold re-scores
    the credited pairs and keeps their forwarding bytes, so the next call runs
    without a full re-score or k_prop_fwd pass (gsx_propagate.hip
    k_prop_count<.., RESCORE>); every call must match the oracle."""
    n, T = 1500, 1
    ov = pc.overlay(n, 6, seed=47, mix_protocols=True, direct_frac=0.02)
    eng, ref = gsx.Engine(T), orc.Oracle(T)
    for be in (eng, ref):
        pc.setup(be, ov, T, 47, disconnect_frac=0.01)
    few = np.random.default_rng(47).choice(n, 25, replace=False)  # a few publishers: their P4 piles up fast
    s0 = eng.scores()
    for k in range(10):
        ms = pc.messages(n, 70 if k % 2 else 40, seed=300 + k, invalid=0.4)
        ms["source"] = few[np.arange(len(ms)) % len(few)]
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, flood_publish=flood_publish, latency_ms=10, seed=9 + k)
        cfg.now_ns = pc.T0 + (2 + k) * pc.S
        res = [be.propagate(ms, cfg, want_results=True) for be in (eng, ref)]
        (go, gh, gf), (wo, wh, wf) = res
        assert go.as_dict() == wo.as_dict(), k
        assert np.array_equal(gh, wh) and np.array_equal(gf, wf), k
        if scores_each or k == 9:
            assert np.array_equal(eng.scores().view(np.uint64), ref.scores().view(np.uint64)), k
    gs, ws = eng.export_state(), ref.export_state()
    for f in abi.STATE_FIELDS:
        assert np.array_equal(gs[f].view(np.uint8), ws[f].view(np.uint8)), f
    s1 = eng.scores()
    assert ((s1 < -300) != (s0 < -300)).sum() > 10  # the credits graylisted senders between calls


@pytest.mark.parametrize("router", [abi.GSX_ROUTER_RANDOMSUB, abi.GSX_ROUTER_GOSSIPSUB])
def test_hub_above_256_peers_matches_oracle(gpu_ok, router):
    """A node with ~600 peers: RandomSub stages its candidate lists over the
    node's own pair range (no degree cap); counters, hops, first deliverers,
    credits and scores == oracle."""
    n, seed = 1500, 77
    ov = pc.with_hub(pc.overlay(n, 5, seed, mix_protocols=True), hub=3, k=600, seed=seed)
    assert np.diff(ov.row_ptr).max() > 256
    ms = pc.messages(n, 100, seed)
    ms["source"][:8] = 3  # the hub publishes too
    cfg = pc.config(router, latency_ms=5, size=50)
    res = []
    for be in (gsx.Engine(1), orc.Oracle(1)):
        pc.setup(be, ov, 1, seed)
        out, hop, frm = be.propagate(ms, cfg, want_results=True)
        res.append((out.as_dict(), hop, frm, be.scores()))
    (go, gh, gf, gsc), (wo, wh, wf, wsc) = res
    assert go == wo
    assert np.array_equal(gh, wh) and np.array_equal(gf, wf)
    assert np.array_equal(gsc.view(np.uint64), wsc.view(np.uint64))
