"""Every BASELINE.json config at its own size on the GPU:

- cfg1  20-peer TestSparseGossipsub-shaped run (tests/sparse_cases.py), engine == oracle,
        every peer receives every message (gossipsub_test.go:43-82);
- cfg2  10k-peer random d=6 overlay, floodsub and gossipsub propagation == oracle;
- cfg3  1M peers x 8 topics: heartbeats (the OpportunisticGraftTicks round and the
        next one) == oracle on the exported state, mesh maintenance, IHAVE gossip,
        backoff, scores bit for bit; and two rounds with the gossip exchange on
        (IWANT, recovery, forwarding, promises, P7) == oracle;
- cfg4  10M-peer overlay on one GPU, floodsub: arrival hops == BFS distances on
        sampled messages, totals consistent (each node reached at most once); and
        the same overlay range-sharded in two (RangeSharded over a local transport)
        == the unsharded engine, hop for hop;
- cfg5  4M peers, 20 % colocated sybils with invalid-message counters: sybils at
        their victims score below GraylistThreshold, and after heartbeats no peer
        whose round-start score was negative is in any mesh, while honest nodes keep
        honest mesh peers (the invariant of gossipsub_test.go:1755-1774).
"""
import numpy as np
import pytest
import torch  # noqa: F401  (initialised before any engine: the shard test's threads use its streams)

import adversarial_cases as ac
import gsx
import heartbeat_cases as hc
import oracle as orc
import propagation_cases as pc
from gsx import abi, synth

pytestmark = pytest.mark.gpu

S = abi.SECOND


def _same(a, b, what):
    assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8)), what


def test_cfg1_sparse_gossipsub_20_peers(gpu_ok):
    import sparse_cases as sc

    g = sc.run(gsx.Engine(1))
    w = sc.run(orc.Oracle(1))
    sc.check(*g)
    assert g[0] == w[0]
    for (go, gh), (wo, wh) in zip(g[1], w[1]):
        assert go == wo
        assert np.array_equal(gh, wh)


@pytest.mark.parametrize("router", [abi.GSX_ROUTER_FLOODSUB, abi.GSX_ROUTER_GOSSIPSUB], ids=["floodsub", "gossipsub"])
@pytest.mark.parametrize("m", [64, 130])
def test_cfg2_10k_peers_matches_oracle(gpu_ok, router, m):
    n, seed = 10_000, 17
    ov = pc.overlay(n, 6, seed, mix_protocols=router == abi.GSX_ROUTER_GOSSIPSUB, direct_frac=0.01)
    ms = pc.messages(n, m, seed)
    cfg = pc.config(router, latency_ms=10)
    res = []
    for be in (gsx.Engine(1), orc.Oracle(1)):
        pc.setup(be, ov, 1, seed, disconnect_frac=0.01)
        out, hop, frm = be.propagate(ms, cfg, want_results=True)
        res.append((out.as_dict(), hop, frm, be.export_state(), be.scores()))
    (go, gh, gf, gs, gsc), (wo, wh, wf, ws, wsc) = res
    assert go == wo
    assert np.array_equal(gh, wh) and np.array_equal(gf, wf)
    for f in abi.STATE_FIELDS:
        _same(gs[f], ws[f], f)
    _same(gsc, wsc, "scores")
    assert go["deliveries"] > 0.9 * m * (n - 1)


def _cfg3_backend(be, ov, T, st):
    be.set_peer_params(synth.bench_peer_params())
    for t in range(T):
        be.set_topic_params(t, synth.spam_test_topic_params())
    be.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                     accept_px_threshold=0, opportunistic_graft_threshold=5))
    be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    be.import_state(st)
    be.set_app_scores(np.zeros(ov.n_pairs))


@pytest.mark.timeout(1200)
def test_cfg3_heartbeat_1m_x_8_matches_oracle(gpu_ok):
    """The bench's cfg3 state: two heartbeats (ticks 60 and 61; 60 is an
    opportunistic-graft round, where every unit with a mesh sorts it) after a
    4-message gossipsub batch fills the message caches."""
    n, T, seed = 1_000_000, 8, synth.SEED
    T0 = pc.T0
    ov = synth.connect_some_overlay(n, d=6, seed=seed)
    e = gsx.Engine(T)
    e.set_peer_params(synth.bench_peer_params())
    for t in range(T):
        e.set_topic_params(t, synth.spam_test_topic_params())
    e.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    e.synthesize_state(abi.SynthSpec(seed=seed, now_ns=T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0,
                                     imd_max_sybil=100.0, p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0,
                                     p_disconnected=0.0, p_absent=0.0, expire_jitter_ns=4 * S, sybil_first_node=n))
    e.set_app_scores(np.zeros(ov.n_pairs))
    e.refresh(T0 + S)
    st = e.export_state()
    o = orc.Oracle(T)
    _cfg3_backend(o, ov, T, st)
    _cfg3_backend(e, ov, T, st)
    del st
    cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, latency_ms=10)
    cfg.now_ns = T0 + 2 * S
    ms = pc.messages(n, 4, 11)
    outs = [be.propagate(ms, cfg)[0].as_dict() for be in (e, o)]
    assert outs[0] == outs[1]
    for k, tick in enumerate((60, 61)):
        now = T0 + (3 + k) * S
        ho = [be.heartbeat(tick, now, seed).as_dict() for be in (e, o)]
        assert ho[0] == ho[1], tick
        assert ho[0]["grafts"] > 0 and ho[0]["ihave_msgs"] > 0
        for f in ("backoff", "scores", "ihave_len", "ihave_digest"):
            a = {"backoff": lambda be: be.export_backoff(), "scores": lambda be: be.scores()}.get(f)
            if a is not None:
                _same(a(e), a(o), (tick, f))
        gl, gd = e.gossip_results()
        wl, wd = o.gossip_results()
        _same(gl, wl, (tick, "ihave_len"))
        _same(gd, wd, (tick, "ihave_digest"))
        del gl, gd, wl, wd
        gs, ws = e.export_state(), o.export_state()
        for f in abi.STATE_FIELDS:
            _same(gs[f], ws[f], (tick, f))
        del gs, ws


@pytest.mark.timeout(1500)
def test_cfg3_gossip_exchange_1m_x_8_matches_oracle(gpu_ok):
    """cfg3 with the gossip exchange on (handleIHave / handleIWant, the
    forwarding of recovered messages, promises, P7): two rounds of a
    64-message gossipsub batch that travels 5 hops (most nodes miss it and
    learn of it by IHAVE, then by the recovering nodes' forwarding) then a
    heartbeat; every round's counters (IWANTs, served, recovered, forwarded,
    broken promises), scores, backoff and state equal the oracle's."""
    import gossip_cases as gc

    n, T, seed = 1_000_000, 8, synth.SEED
    ov = synth.connect_some_overlay(n, d=6, seed=seed)
    e = gsx.Engine(T)
    e.set_peer_params(synth.bench_peer_params())
    for t in range(T):
        e.set_topic_params(t, synth.spam_test_topic_params())
    e.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    e.synthesize_state(abi.SynthSpec(seed=seed, now_ns=pc.T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0,
                                     imd_max_sybil=100.0, p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0,
                                     p_disconnected=0.0, p_absent=0.0, expire_jitter_ns=4 * S, sybil_first_node=n))
    e.set_app_scores(np.zeros(ov.n_pairs))
    e.refresh(pc.T0 + S)
    st = e.export_state()
    o = orc.Oracle(T)
    _cfg3_backend(o, ov, T, st)
    _cfg3_backend(e, ov, T, st)
    del st
    gp = gc.params(iwant_followup_ns=S // 2)  # promises of round k break at round k + 1 (P7 within the run)
    for be in (e, o):
        be.set_gossipsub_params(gp)
    tot = {}
    for k in range(2):
        now = pc.T0 + (2 + k) * S
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % 2, max_hops=5, latency_ms=10, seed=7 + k)
        cfg.now_ns = now
        ms = pc.messages(n, 64, 100 + k)
        outs = [be.propagate(ms, cfg)[0].as_dict() for be in (e, o)]
        assert outs[0] == outs[1], k
        ho = [be.heartbeat(61 + k, now + 500 * abi.MILLISECOND, seed).as_dict() for be in (e, o)]
        assert ho[0] == ho[1], (k, {x: (ho[0][x], ho[1][x]) for x in ho[0] if ho[0][x] != ho[1][x]})
        for x, v in ho[0].items():
            tot[x] = tot.get(x, 0) + v
        _same(e.scores(), o.scores(), (k, "scores"))
        _same(e.export_backoff(), o.export_backoff(), (k, "backoff"))
        gs, ws = e.export_state(), o.export_state()
        for f in abi.STATE_FIELDS:
            _same(gs[f], ws[f], (k, f))
        del gs, ws
    assert tot["iwant_msgs"] > 0 and tot["gossip_delivered"] > 0 and tot["broken_promises"] > 0, tot
    assert tot["fwd_delivered"] > 0 and tot["fwd_duplicates"] > 0, tot


@pytest.mark.timeout(1500)
def test_cfg3_sharded_gossip_exchange_1m_matches_single_engine(gpu_ok):
    """The gossip exchange on range shards at cfg3's size: 1M peers in two
    RangeSharded shards (lock-step threads on one GPU) against the unsharded
    engine, through propagate -> heartbeat rounds whose gossip windows hold
    more ids than the reference's MaxIHaveLength of 5000 (2,048-message
    batches that travel 3 hops), so most IHAVE lists are truncated per target
    and cross the shards as subsets.  Counters summed over the ranks, scores,
    backoff and records of every node equal the single engine's."""
    import gossip_cases as gc
    from gsx import shard

    n, T, seed, world = 1_000_000, 2, synth.SEED, 2
    ov = synth.connect_some_overlay(n, d=6, seed=seed)
    spec = abi.SynthSpec(seed=seed, now_ns=pc.T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0, imd_max_sybil=100.0,
                         p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0, p_disconnected=0.0, p_absent=0.0,
                         expire_jitter_ns=4 * S, sybil_first_node=n)
    gp = gc.params(iwant_followup_ns=S // 2)
    full = gsx.Engine(T)
    full.set_peer_params(synth.bench_peer_params())
    for t in range(T):
        full.set_topic_params(t, synth.spam_test_topic_params())
    full.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                       accept_px_threshold=0, opportunistic_graft_threshold=5))
    full.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    full.synthesize_state(spec)
    full.set_app_scores(np.zeros(ov.n_pairs))
    full.refresh(pc.T0 + S)
    full.set_gossipsub_params(gp)
    st = full.export_state()
    E = ov.n_pairs
    rank_lo = synth.shard_ranges(n, world)
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
        sh = synth.shard_of(ov, lo, hi)
        e = gsx.Engine(T)
        e.set_peer_params(synth.bench_peer_params())
        for t in range(T):
            e.set_topic_params(t, synth.spam_test_topic_params())
        e.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                        accept_px_threshold=0, opportunistic_graft_threshold=5))
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        sl = {}
        for f in abi.STATE_FIELDS:
            x = st[f]
            sl[f] = x.reshape(T, E)[:, a:b].reshape(-1).copy() if f in abi.RECORD_FIELDS else x[a:b].copy()
        sl["last_refresh_ns"] = st["last_refresh_ns"]
        e.import_state(sl)
        e.set_app_scores(np.zeros(b - a))
        e.set_gossipsub_params(gp)
        engines.append((e, a, b, lo, hi))
        del sh, sl
    del st
    runners = shard.run_local(world, "cuda:0", lambda tp, e: shard.RangeSharded(e, rank_lo, tp),
                              [(x[0],) for x in engines])
    tot, truncated = {}, 0
    for k in range(4):
        now = pc.T0 + (2 + k) * S
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=0, max_hops=3, latency_ms=10, seed=7 + k)
        cfg.now_ns = now
        ms = pc.messages(n, 2048, 100 + k)
        want = full.propagate(ms, cfg)[0].as_dict()
        res = shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.propagate(ms, cfg))[1],
                              [(r,) for r in runners])
        for x in ("deliveries", "duplicates", "transmissions", "hops"):
            assert res[0][1][x] == want[x], (k, x)
        tick, hn = 61 + k, now + 500 * abi.MILLISECOND
        want = full.heartbeat(tick, hn, seed).as_dict()
        res = shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.heartbeat(tick, hn, seed))[1],
                              [(r,) for r in runners])
        assert res[0][1] == want, (k, {x: (res[0][1][x], want[x]) for x in want if res[0][1][x] != want[x]})
        for x, v in want.items():
            tot[x] = tot.get(x, 0) + v
        sc, bo = full.scores(), np.asarray(full.export_backoff()).reshape(T, E)
        il = np.asarray(full.gossip_results()[0]).reshape(T, E)
        fs = full.export_state()
        for (e, a, b, lo, hi) in engines:
            _same(e.scores(), sc[a:b], (k, "scores"))
            _same(np.asarray(e.export_backoff()).reshape(T, b - a), bo[:, a:b], (k, "backoff"))
            es = e.export_state()
            for f in abi.STATE_FIELDS:
                w = fs[f].reshape(T, E)[:, a:b].reshape(-1) if f in abi.RECORD_FIELDS else fs[f][a:b]
                _same(es[f], w, (k, f))
            del es
            cross = (ov.col[a:b] < lo) | (ov.col[a:b] >= hi)
            truncated += int(((il[:, a:b] == gp.max_ihave_length) & cross[None, :]).sum())
        del fs
    assert tot["iwant_msgs"] > 0 and tot["gossip_delivered"] > 0 and tot["fwd_delivered"] > 0, tot
    assert truncated > 0


def _bfs(row_ptr, col, src):
    """Level-synchronous BFS over a CSR overlay (numpy): hop distance per node, -1 unreached."""
    n = len(row_ptr) - 1
    dist = np.full(n, -1, dtype=np.int64)
    dist[src] = 0
    front = np.array([src], dtype=np.int64)
    d = 0
    while len(front):
        d += 1
        starts, ends = row_ptr[front], row_ptr[front + 1]
        lens = ends - starts
        idx = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        nb = np.unique(col[idx])
        nb = nb[dist[nb] < 0]
        dist[nb] = d
        front = nb
    return dist


@pytest.mark.timeout(1200)
def test_cfg4_10m_floodsub_properties(gpu_ok):
    n, seed = 10_000_000, synth.SEED + 1
    ov = synth.connect_some_overlay(n, d=6, seed=seed)
    e = gsx.Engine(1)
    e.set_peer_params(synth.bench_peer_params())
    e.set_topic_params(0, synth.spam_test_topic_params())
    e.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    e.synthesize_state(abi.SynthSpec(seed=seed, now_ns=pc.T0, fmd_max=10, mmd_max=10, mfp_max=1, imd_max_sybil=0,
                                     p_in_mesh=0.5, graft_window_ns=abi.HOUR, bp_max=0, p_disconnected=0,
                                     p_absent=0, expire_jitter_ns=0, sybil_first_node=n))
    e.set_prop_tracking(False)
    ms = pc.messages(n, 64, 12)
    out, hop, _ = e.propagate(ms, pc.config(abi.GSX_ROUTER_FLOODSUB, credit=0), want_results=True)
    reached = hop != 0xFF
    assert out.deliveries == int(reached.sum()) - len(ms)  # each (node, message) reached at most once
    assert out.transmissions == out.deliveries + out.duplicates
    assert reached.mean() > 0.999
    for k in range(2):
        dist = _bfs(ov.row_ptr, ov.col.astype(np.int64), int(ms["source"][k]))
        r = dist >= 0
        assert np.array_equal(reached[k], r)
        assert np.array_equal(hop[k][r].astype(np.int64), dist[r])


@pytest.mark.timeout(1200)
def test_cfg4_10m_range_sharded_matches_single_engine(gpu_ok):
    """cfg4's own layout: the 10M overlay split into two RangeSharded shards
    (gsx/shard.py, the per-hop compacted frontier exchange) run as lock-step
    threads on one GPU, BASELINE's 64-message floodsub batch.  The stitched
    arrival hops equal the unsharded engine's, the totals equal, and sampled
    messages' hops are BFS distances."""
    from gsx import shard

    n, seed, world = 10_000_000, synth.SEED + 1, 2
    ov = synth.connect_some_overlay(n, d=6, seed=seed)
    spec = abi.SynthSpec(seed=seed, now_ns=pc.T0, fmd_max=10, mmd_max=10, mfp_max=1, imd_max_sybil=0, p_in_mesh=0.5,
                         graft_window_ns=abi.HOUR, bp_max=0, p_disconnected=0, p_absent=0, expire_jitter_ns=0,
                         sybil_first_node=n)

    def params(e):
        e.set_peer_params(synth.bench_peer_params())
        e.set_topic_params(0, synth.spam_test_topic_params())

    ms = pc.messages(n, 64, 12)
    cfg = pc.config(abi.GSX_ROUTER_FLOODSUB, credit=0)
    full = gsx.Engine(1)
    params(full)
    full.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    full.synthesize_state(spec)
    full.set_prop_tracking(False)
    out, hop, _ = full.propagate(ms, cfg, want_results=True)
    full.close()
    rank_lo = synth.shard_ranges(n, world)
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        sh = synth.shard_of(ov, lo, hi)
        e = gsx.Engine(1)
        params(e)
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.synthesize_state(spec)  # (every pair present and connected: floodsub without credits reads nothing else)
        e.set_prop_tracking(False)
        engines.append(e)
        del sh
    res = shard.run_local(world, "cuda:0", lambda tp, e: shard.RangeSharded(e, rank_lo, tp).propagate(ms, cfg),
                          [(e,) for e in engines])
    tot, want = res[0][1], out.as_dict()
    for k in ("deliveries", "duplicates", "transmissions", "hops", "hop_deliveries"):
        assert tot[k] == want[k], k
    for k, e in enumerate(engines):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        h, _ = e.prop_results(len(ms))
        assert np.array_equal(h, hop[:, lo:hi]), (k, np.argwhere(h != hop[:, lo:hi])[:5])
        e.close()
    reached = hop != 0xFF
    assert out.deliveries == int(reached.sum()) - len(ms) and reached.mean() > 0.999
    for k in range(2):
        dist = _bfs(ov.row_ptr, ov.col.astype(np.int64), int(ms["source"][k]))
        r = dist >= 0
        assert np.array_equal(reached[k], r)
        assert np.array_equal(hop[k][r].astype(np.int64), dist[r])


@pytest.mark.timeout(1200)
def test_cfg4_10m_gossipsub_credits_range_sharded(gpu_ok):
    """The router the cfg4 bench leg times (bench.py prop_engine/prop_config):
    gossipsub over the synthesized mesh, P2/P3 credits on at delivery time,
    per-pair first-receipt counts (no first-deliverer rows), BASELINE's
    64-message batch on the 10M overlay.  Two RangeSharded shards holding the
    single engine's state slices equal it bit for bit after the batch: arrival
    hops, totals, every pair's state (the credited P2/P3 counters among them)
    and every score."""
    from gsx import shard

    n, seed, world, T = 10_000_000, synth.SEED + 1, 2, 1
    ov = synth.connect_some_overlay(n, d=6, seed=seed)
    th = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                        accept_px_threshold=0, opportunistic_graft_threshold=0)

    def params(e):
        e.set_peer_params(synth.bench_peer_params())
        e.set_topic_params(0, synth.spam_test_topic_params())
        e.set_thresholds(th)
        e.set_prop_tracking(False)

    full = gsx.Engine(T)
    params(full)
    full.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    full.synthesize_state(
        abi.SynthSpec(seed=seed, now_ns=pc.T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0, imd_max_sybil=100.0,
                      p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0, p_disconnected=0.0, p_absent=0.0,
                      expire_jitter_ns=4 * abi.SECOND, sybil_first_node=n))
    full.set_app_scores(np.zeros(ov.n_pairs))
    full.refresh(pc.T0 + S)
    st0 = full.export_state()
    ms = pc.messages(n, 64, 12)
    cfg = abi.PropConfig(router=abi.GSX_ROUTER_GOSSIPSUB, topic=0, flood_publish=0, max_hops=40,
                         hop_latency_ns=10 * abi.MILLISECOND, now_ns=pc.T0 + 2 * S,
                         credit_scores=abi.GSX_CREDIT_NOW, randomsub_size=n, seed=synth.SEED)
    out, hop, _ = full.propagate(ms, cfg, want_results=True)
    st1, sc1 = full.export_state(), full.scores()
    full.close()
    E = ov.n_pairs

    def part(st, a, b):
        p = {f: (st[f].reshape(T, E)[:, a:b].reshape(-1).copy() if f in abi.RECORD_FIELDS else st[f][a:b].copy())
             for f in abi.STATE_FIELDS}
        p["last_refresh_ns"] = st["last_refresh_ns"]
        return p

    rank_lo = synth.shard_ranges(n, world)
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
        sh = synth.shard_of(ov, lo, hi)
        e = gsx.Engine(T)
        params(e)
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.import_state(part(st0, a, b))
        e.set_app_scores(np.zeros(b - a))
        engines.append((e, a, b))
        del sh
    del st0
    res = shard.run_local(world, "cuda:0", lambda tp, e: shard.RangeSharded(e, rank_lo, tp).propagate(ms, cfg),
                          [(e,) for e, _, _ in engines])
    tot, want = res[0][1], out.as_dict()
    for k in ("deliveries", "duplicates", "transmissions", "hops", "hop_deliveries", "graylisted"):
        assert tot[k] == want[k], k
    assert want["deliveries"] > 0.9 * len(ms) * n * 0.5
    for k, (e, a, b) in enumerate(engines):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        h, _ = e.prop_results(len(ms))
        assert np.array_equal(h, hop[:, lo:hi]), (k, np.argwhere(h != hop[:, lo:hi])[:5])
        st, want_st = e.export_state(), part(st1, a, b)
        for fld in abi.STATE_FIELDS:
            assert np.array_equal(st[fld].view(np.uint8), want_st[fld].view(np.uint8)), (k, fld)
        assert np.array_equal(e.scores().view(np.uint64), sc1[a:b].view(np.uint64)), k
        e.close()


@pytest.mark.timeout(1200)
def test_cfg5_4m_adversarial_properties(gpu_ok):
    n = 4_000_000
    e = gsx.Engine(1)
    ov = ac.setup(e, n, seed=23)
    sc = e.scores()
    syb = ac.sybil_pairs(ov)
    vic = ac.victim_pairs(ov)
    th = ac.TH.graylist_threshold
    assert (sc[vic & syb] < th).all()  # P6 (colocation) + P4 (invalid spam) graylist the attackers
    assert (sc[~syb] >= th).mean() > 0.75
    obs = ov.pair_observer()
    honest_node = ~ov.sybil
    # the reference test's honest peers score >= 0 (AppSpecificScore 0 and good
    # deliveries, gossipsub_test.go:1680-1700): give every honest pair a positive
    # application score, the sybils keep theirs (P6 + P4 negative)
    e.set_app_scores(np.where(syb, 0.0, 1000.0))
    for k, tick in enumerate((59, 60)):
        start = e.scores()
        e.heartbeat(tick, ac.T0 + (2 + k) * S, 9)
        e.refresh(ac.T0 + (2 + k) * S + 500 * abi.MILLISECOND)
        inm = (e.export_state()["rec_flags"] & abi.GSX_REC_IN_MESH) != 0
        # (A) prunes negative-score mesh peers and grafts only score >= 0; (B)
        # accepts GRAFTs only from score >= 0 peers: a peer scoring below zero at
        # the round start is in nobody's mesh at its end
        assert not (inm & (start < 0)).any(), tick
    # honest observers keep honest mesh peers (gossipsub_test.go:1755-1774: >= 3)
    honest_links = inm & ~syb & honest_node[obs]
    per_node = np.bincount(obs[honest_links], minlength=ov.n)
    has3 = np.bincount(obs[~syb & honest_node[obs] & (start >= 0)], minlength=ov.n) >= 3
    frac = (per_node[honest_node & has3] >= 3).mean()
    assert frac > 0.99, frac
    assert not (inm & syb & vic).any()  # no colocated sybil stays in a victim's mesh
