"""Multi-GPU propagation drivers (gsx/shard.py) on one GPU: several engines,
one per shard (or replica), run as lock-step threads that exchange through
device copies instead of RCCL.  Every per-node result, counter, credited
score state and score must equal the single-engine run bit for bit (which
test_gpu_propagation.py pins to the oracle)."""
import numpy as np
import pytest
import torch  # noqa: F401  (imported on the main thread before the shard threads use it)

import gsx
import propagation_cases as pc
from gsx import abi, shard, synth

pytestmark = pytest.mark.gpu


def _params(e, T, window_ms=25):
    e.set_peer_params(synth.bench_peer_params())
    for t in range(T):
        tp = synth.spam_test_topic_params()
        tp.mesh_message_deliveries_window_ns = int(window_ms * abi.MILLISECOND)
        e.set_topic_params(t, tp)
    e.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                    accept_px_threshold=0, opportunistic_graft_threshold=0))


def _slice_state(st, T, E, a, b):
    out = {}
    for f in abi.STATE_FIELDS:
        x = st[f]
        out[f] = x.reshape(T, E)[:, a:b].reshape(-1).copy() if f in abi.RECORD_FIELDS else x[a:b].copy()
    out["last_refresh_ns"] = st["last_refresh_ns"]
    return out


CASES = [
    # world, n, d, T, router, flood_publish, m, mix, disconnect, compact
    (2, 1500, 4, 1, abi.GSX_ROUTER_FLOODSUB, 0, 64, False, 0.02, False),
    (2, 1500, 4, 1, abi.GSX_ROUTER_FLOODSUB, 0, 64, False, 0.02, True),
    (2, 2000, 6, 2, abi.GSX_ROUTER_GOSSIPSUB, 0, 200, True, 0.03, True),
    (3, 1800, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 100, True, 0.0, False),
    (3, 1800, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 100, True, 0.0, True),
    (4, 1600, 4, 1, abi.GSX_ROUTER_RANDOMSUB, 0, 64, True, 0.02, True),
    (2, 1500, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 1024, True, 0.02, True),
    (3, 1200, 4, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 500, True, 0.0, False),
    # shards without first-deliverer rows (counts only)
    (2, 2000, 6, 2, abi.GSX_ROUTER_GOSSIPSUB, 0, 200, True, 0.03, "compact-counts"),
    (3, 1800, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 1024, True, 0.02, "dense-counts"),
    (2, 1500, 4, 1, abi.GSX_ROUTER_FLOODSUB, 0, 300, False, 0.02, "compact-counts"),
    # validation outcomes (dropped / rejected messages) and a validation delay
    (3, 1800, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 300, True, 0.02, "compact-invalid"),
    (2, 1500, 5, 2, abi.GSX_ROUTER_GOSSIPSUB, 1, 200, True, 0.02, "dense-counts-invalid"),
    (2, 1600, 4, 1, abi.GSX_ROUTER_RANDOMSUB, 0, 100, True, 0.02, "compact-invalid"),
    # batches cut short by max_hops (the last hop still delivers), rows of several chunks per lane
    (2, 1500, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 1100, True, 0.02, "compact-counts-cut"),
    (3, 1200, 4, 1, abi.GSX_ROUTER_FLOODSUB, 0, 2048, False, 0.0, "compact-cut"),
    # every duplicate inside the P3 window ("late"): the shards run the lean hop
    # kernels (k_prop_hop_fast1 / k_prop_hop_fast, SH instance: remote rows from
    # the halo, their duplicates counted per hop, graylisted senders dropped)
    (2, 1500, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 64, True, 0.02, "compact-counts-late"),
    (3, 1800, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 40, True, 0.02, "dense-counts-late"),
    (4, 1600, 4, 1, abi.GSX_ROUTER_FLOODSUB, 0, 64, False, 0.02, "compact-counts-invalid-late"),
    (2, 1500, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 64, True, 0.02, "compact-counts-late-cut"),
    (2, 2000, 6, 2, abi.GSX_ROUTER_GOSSIPSUB, 0, 1024, True, 0.03, "compact-counts-late"),
    (3, 1500, 4, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 200, True, 0.02, "compact-counts-invalid-late"),
    (3, 1200, 4, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 500, True, 0.0, "dense-counts-late"),
    (2, 1500, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 0, 1100, True, 0.02, "compact-counts-late-cut"),
    (2, 1500, 5, 1, abi.GSX_ROUTER_GOSSIPSUB, 1, 256, True, 0.02, "compact-counts-invalid-late"),
]


@pytest.mark.parametrize("case", CASES,
                         ids=[f"w{c[0]}-r{c[4]}-m{c[6]}-{c[9] if isinstance(c[9], str) else ('compact' if c[9] else 'dense')}"
                              for c in CASES])
def test_range_sharded_matches_single_engine(gpu_ok, case):
    world, n, d, T, router, fp, m, mix, disc, compact = case
    track, invalid, delay, max_hops, window_ms = True, 0.0, 0.0, 40, 25
    if isinstance(compact, str):  # "<exchange>[-counts][-invalid][-late][-cut]"
        track = "counts" not in compact
        if "invalid" in compact:  # messages validation drops, and a validation delay
            invalid, delay = 0.25, 3.0
        if "cut" in compact:
            max_hops = 3
        if "late" in compact:  # a 5-minute P3 window: every duplicate inside it
            window_ms = 300_000
        compact = compact.startswith("compact")
    seed = 3 * n + m
    ov = pc.overlay(n, d, seed, mix_protocols=mix, direct_frac=0.03 if mix else 0.0)
    msgs = pc.messages(n, m, seed, invalid=invalid)
    cfg = pc.config(router, topic=T - 1, flood_publish=fp, size=60, delay_ms=delay, max_hops=max_hops)
    full = gsx.Engine(T)
    app = pc.setup(full, ov, T, seed, disconnect_frac=disc)
    if window_ms != 25:
        _params(full, T, window_ms)
    st0 = full.export_state()
    out, hop, frm = full.propagate(msgs, cfg, want_results=True)
    st1, sc1 = full.export_state(), full.scores()

    rank_lo = synth.shard_ranges(n, world)
    E = ov.n_pairs
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        sh = synth.shard_of(ov, lo, hi)
        a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
        e = gsx.Engine(T)
        _params(e, T, window_ms)
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.import_state(_slice_state(st0, T, E, a, b))
        e.set_app_scores(app[a:b])
        e.set_prop_tracking(track)
        engines.append((e, a, b))

    def run(tp, e):
        rs = shard.RangeSharded(e, rank_lo, tp, compact=compact)
        return rs.propagate(msgs, cfg)

    res = shard.run_local(world, "cuda:0", run, [(e,) for e, _, _ in engines])
    tot = res[0][1]
    want = out.as_dict()
    for k in ("deliveries", "duplicates", "transmissions", "hops", "hop_deliveries", "rejected", "ignored", "graylisted"):
        assert tot[k] == want[k], k
    assert tot["new_words"] == out.new_words
    # edge_sends is the traffic term of the exchange: a shard packs a row for a
    # remote receiver that graylists the sender (the copies cross xGMI and are
    # dropped there), while one engine never gathers such a row
    if want["graylisted"]:
        assert tot["edge_sends"] >= out.edge_sends
    else:
        assert tot["edge_sends"] == out.edge_sends
    for k, (e, a, b) in enumerate(engines):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        h, f = e.prop_results(m)
        assert np.array_equal(h, hop[:, lo:hi]), (k, np.argwhere(h != hop[:, lo:hi])[:5])
        if track:
            assert np.array_equal(f, frm[:, lo:hi]), (k, np.argwhere(f != frm[:, lo:hi])[:5])
        st = e.export_state()
        want_st = _slice_state(st1, T, E, a, b)
        for fld in abi.STATE_FIELDS:
            assert np.array_equal(st[fld].view(np.uint8), want_st[fld].view(np.uint8)), (k, fld)
        assert np.array_equal(e.scores().view(np.uint64), sc1[a:b].view(np.uint64)), k
    assert want["deliveries"] > 0


@pytest.mark.parametrize("world,invalid", [(2, 0.0), (3, 0.0), (3, 0.2)])
def test_message_parallel_matches_single_engine(gpu_ok, world, invalid):
    n, d, T, m = 3000, 6, 1, 300
    seed = 17 + world
    ov = pc.overlay(n, d, seed, mix_protocols=True, direct_frac=0.02)
    msgs = pc.messages(n, m, seed, invalid=invalid)
    cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, latency_ms=4)
    full = gsx.Engine(T)
    pc.setup(full, ov, T, seed, disconnect_frac=0.02)
    out = full.propagate(msgs, cfg)[0]
    st1, sc1 = full.export_state(), full.scores()
    reps = []
    for _ in range(world):
        e = gsx.Engine(T)
        pc.setup(e, ov, T, seed, disconnect_frac=0.02)
        reps.append(e)

    def run(tp, e):
        return shard.MessageParallel(e, tp).propagate(msgs, cfg)

    res = shard.run_local(world, "cuda:0", run, [(e,) for e in reps])
    tot = res[0][1]
    want = out.as_dict()
    for k in ("deliveries", "duplicates", "transmissions", "hops", "hop_deliveries", "rejected", "ignored", "graylisted"):
        assert tot[k] == want[k], k
    for e in reps:
        st = e.export_state()
        for fld in abi.STATE_FIELDS:
            assert np.array_equal(st[fld].view(np.uint8), st1[fld].view(np.uint8)), fld
        assert np.array_equal(e.scores().view(np.uint64), sc1.view(np.uint64))


@pytest.mark.parametrize("m", [130, 40])
def test_stepped_api_equals_propagate(gpu_ok, m):
    """gsx_prop_begin + steps + end on an unsharded engine == gsx_propagate;
    deferred credits folded later == credits folded at once (m = 40: one-word
    rows, k_prop_hop_fast1 with flast kept every hop)."""
    n, T = 2500, 1
    ov = pc.overlay(n, 5, 5, mix_protocols=True)
    msgs = pc.messages(n, m, 5)
    cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, latency_ms=7)
    a, b = gsx.Engine(T), gsx.Engine(T)
    for e in (a, b):
        pc.setup(e, ov, T, 5)
    oa = a.propagate(msgs, cfg)[0]
    cfg_d = pc.config(abi.GSX_ROUTER_GOSSIPSUB, latency_ms=7, credit=abi.GSX_CREDIT_DEFER)
    b.prop_begin(msgs, cfg_d)
    for _ in range(cfg_d.max_hops):
        b.prop_step(0)
    ob = b.prop_end()
    assert oa.as_dict() == ob.as_dict()
    first = np.zeros(ov.n_pairs, dtype=np.uint32)
    dup = np.zeros(ov.n_pairs, dtype=np.uint32)
    b.pending_credits(first.ctypes.data, dup.ctypes.data)
    assert first.sum() == oa.deliveries
    b.fold_credits()
    assert np.array_equal(a.scores().view(np.uint64), b.scores().view(np.uint64))
    ha, fa = a.prop_results(m)
    hb, fb = b.prop_results(m)
    assert np.array_equal(ha, hb) and np.array_equal(fa, fb)


def _slice_te(x, T, E, a, b):
    return np.asarray(x).reshape(T, E)[:, a:b].reshape(-1)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_heartbeat_matches_single_engine(gpu_ok, world):
    """Heartbeat rounds on range shards (GRAFT/PRUNE words and PRUNE answers of
    cross-shard pairs exchanged between the steps) == one engine, including
    the IHAVE gossip of a propagated batch; counters summed over ranks."""
    import heartbeat_cases as hc

    n, d, T, seed = 1500, 7, 2, 41
    ov = pc.overlay(n, d, seed, mix_protocols=True, direct_frac=0.02)
    full = gsx.Engine(T)
    app = pc.setup(full, ov, T, seed, mesh_degree=9, disconnect_frac=0.02)
    st0 = full.export_state()
    E = ov.n_pairs
    rank_lo = synth.shard_ranges(n, world)
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        sh = synth.shard_of(ov, lo, hi)
        a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
        e = gsx.Engine(T)
        _params(e, T)
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.import_state(_slice_state(st0, T, E, a, b))
        e.set_app_scores(app[a:b])
        engines.append((e, a, b))
    runners = shard.run_local(world, "cuda:0", lambda tp, e: shard.RangeSharded(e, rank_lo, tp),
                              [(e,) for e, _, _ in engines])
    msgs = pc.messages(n, 100, seed)
    for k in range(3):
        tick, now = 59 + k, pc.T0 + (3 + k) * abi.SECOND
        want = full.heartbeat(tick, now, seed).as_dict()
        res = shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.heartbeat(tick, now, seed))[1],
                              [(r,) for r in runners])
        assert res[0][1] == want, (k, res[0][1], want)
        snap = hc.snapshot(full)
        for (e, a, b) in engines:
            got = hc.snapshot(e)
            for f in abi.STATE_FIELDS:
                w = _slice_state(snap, T, E, a, b)[f]
                assert np.array_equal(got[f].view(np.uint8), w.view(np.uint8)), (k, f)
            for f in ("backoff", "ihave_len", "ihave_digest"):
                assert np.array_equal(np.asarray(got[f]).reshape(-1), _slice_te(snap[f], T, E, a, b)), (k, f)
            assert np.array_equal(got["scores"].view(np.uint64), snap["scores"][a:b].view(np.uint64)), k
        if k == 0:  # a gossipsub batch for the next rounds' IHAVEs (every engine caches what it saw)
            cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=0, latency_ms=5)
            full.propagate(msgs, cfg)
            shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.propagate(msgs, cfg))[1],
                            [(r,) for r in runners])
    assert want["grafts"] + want["prunes"] > 0


@pytest.mark.parametrize("world,invalid,T,max_ihave,m,window",
                         [(2, 0.0, 2, 5000, 24, None), (3, 0.2, 2, 5000, 24, None), (2, 0.0, 1, 5000, 24, None),
                          (2, 0.0, 2, 20, 24, None), (3, 0.2, 1, 20, 24, None), (3, 0.0, 1, 5000, 2600, None),
                          (2, 0.0, 2, 5000, 24, 892), (3, 0.2, 1, 20, 24, 1000)],
                         ids=["w2-T2", "w3-T2-invalid", "w2-T1", "w2-T2-trunc20", "w3-T1-trunc20-invalid",
                              "w3-T1-trunc5000", "w2-T2-window-hop1_2", "w3-T1-trunc20-window-one_round"])
def test_sharded_heartbeat_exchange_matches_single_engine(gpu_ok, world, invalid, T, max_ihave, m, window):
    """The gossip exchange on range shards (gsx_gx_*: IHAVE bits and answer
    bits of cross-shard pairs, the senders' cache rows, the forwarding of
    recovered messages hop by hop with frontier entries): rounds of a
    heartbeat with the exchange on, then a gossipsub batch that travels two
    hops (most nodes miss it and recover it by IHAVE / IWANT and the
    recovering nodes' forwarding), == one engine: counters summed over ranks,
    every node's records, backoff, IHAVEs, scores and cached ids.  The trunc
    cases hold more ids in the gossip window than MaxIHaveLength (20, or the
    reference's 5000 with 2,600-message batches): every target gets its own
    subset (gossipsub.go:1708-1720), which crosses the shards as masked rows.
    The window cases put the P3 window boundary between arrival hops / recovery
    rounds (per-node validation times): the senders' inside rows travel with
    their cache rows for the hop-1 back-sends."""
    import gossip_cases as gc
    import heartbeat_cases as hc

    n, d, seed = 1200, 6, 47
    ov = pc.overlay(n, d, seed)
    full = gsx.Engine(T)
    app = pc.setup(full, ov, T, seed, mesh_degree=6)
    if window is not None:
        _params(full, T, window)
    gp = gc.params(max_ihave_length=max_ihave)
    full.set_gossipsub_params(gp)
    st0 = full.export_state()
    E = ov.n_pairs
    rank_lo = synth.shard_ranges(n, world)
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        sh = synth.shard_of(ov, lo, hi)
        a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
        e = gsx.Engine(T)
        _params(e, T, 25 if window is None else window)
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.import_state(_slice_state(st0, T, E, a, b))
        e.set_app_scores(app[a:b])
        e.set_gossipsub_params(gp)
        engines.append((e, a, b, lo, hi))
    runners = shard.run_local(world, "cuda:0", lambda tp, e: shard.RangeSharded(e, rank_lo, tp),
                              [(x[0],) for x in engines])
    tot = {}
    truncated = 0
    for k in range(6):
        tick, now = 1 + k, pc.T0 + (3 + k) * abi.SECOND
        want = full.heartbeat(tick, now, seed * 31 + 7).as_dict()
        res = shard.run_local(world, "cuda:0",
                              lambda tp, r: (setattr(r, "tp", tp), r.heartbeat(tick, now, seed * 31 + 7))[1],
                              [(r,) for r in runners])
        assert res[0][1] == want, (k, {x: (res[0][1][x], want[x]) for x in want if res[0][1][x] != want[x]})
        for x, v in want.items():
            tot[x] = tot.get(x, 0) + v
        snap = hc.snapshot(full)
        il = np.asarray(snap["ihave_len"]).reshape(T, E)
        for (e, a, b, lo, hi) in engines:
            got = hc.snapshot(e)
            for f in abi.STATE_FIELDS:
                w = _slice_state(snap, T, E, a, b)[f]
                assert np.array_equal(got[f].view(np.uint8), w.view(np.uint8)), (k, f)
            for f in ("backoff", "ihave_len", "ihave_digest"):
                assert np.array_equal(np.asarray(got[f]).reshape(-1), _slice_te(snap[f], T, E, a, b)), (k, f)
            assert np.array_equal(got["scores"].view(np.uint64), snap["scores"][a:b].view(np.uint64)), k
            for v in range(lo, hi, 37):  # the caches (recovered copies Put)
                assert sorted(e.mcache_ids(v - lo, abi.GSX_ANY_TOPIC, 5).tolist()) == \
                    sorted(full.mcache_ids(v, abi.GSX_ANY_TOPIC, 5).tolist()), (k, v)
            # truncated lists sent over this rank's cross-shard pairs (the case under test)
            cross = (ov.col[a:b] < lo) | (ov.col[a:b] >= hi)
            truncated += int(((il[:, a:b] == max_ihave) & cross[None, :]).sum())
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, max_hops=2, latency_ms=5, seed=seed + k)
        cfg.now_ns = now + 100 * abi.MILLISECOND
        ms = pc.messages(n, m, seed + 1000 * k, invalid=invalid)
        full.propagate(ms, cfg)
        shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.propagate(ms, cfg))[1],
                        [(r,) for r in runners])
        full.refresh(now + 500 * abi.MILLISECOND)
        for (e, _, _, _, _) in engines:
            e.refresh(now + 500 * abi.MILLISECOND)
    assert tot["iwant_msgs"] > 0 and tot["gossip_delivered"] > 0 and tot["fwd_delivered"] > 0, tot
    if max_ihave < 5000 or m > 1000:
        assert truncated > 0


@pytest.mark.parametrize("world,invalid,window", [(2, 0.0, None), (3, 0.2, None), (2, 0.0, 892)])
def test_message_parallel_heartbeat_matches_single_engine(gpu_ok, world, invalid, window):
    """Message-parallel replicas through propagate -> heartbeat cycles with the
    gossip exchange on: every replica propagates its block, the cache blocks
    are all-gathered and Put back whole (gsx_mcache_put, k_mc_merge), the
    credits are summed and folded, and every replica runs the whole round.
    Counters, records, backoff, scores, IHAVEs and cached ids == one engine."""
    import gossip_cases as gc

    kw = dict(n=1500, ticks=4, msgs=150, invalid=invalid)
    if window is not None:  # the window boundary between arrival hops: the blocks carry their code planes
        kw.update(window_ms=window, hops=3)
    _, want_outs, want_snaps, want_cached = gc.exchange_run(gsx.Engine(2), **kw)
    assert sum(o["iwant_msgs"] for o in want_outs) > 0 and sum(o["gossip_delivered"] for o in want_outs) > 0

    def run(tp, e):
        r = shard.MessageParallel(e, tp)
        _, outs, snaps, cached = gc.exchange_run(e, runner=r, **kw)
        return outs, snaps, cached, r.gathered_bytes

    res = shard.run_local(world, "cuda:0", run, [(gsx.Engine(2),) for _ in range(world)])
    for rank, (outs, snaps, cached, gathered) in enumerate(res):
        assert outs == want_outs, rank
        for k, (a, b) in enumerate(zip(snaps, want_snaps)):
            for f in a:
                assert np.array_equal(np.asarray(a[f]).reshape(-1).view(np.uint8),
                                      np.asarray(b[f]).reshape(-1).view(np.uint8)), (rank, k, f)
        for v in range(0, len(cached), 7):
            assert np.array_equal(np.sort(cached[v]), np.sort(want_cached[v])), (rank, v)
        assert gathered > 0


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_heartbeat_peer_exchange_matches_single_engine(gpu_ok, world):
    """WithPeerExchange on range shards: the PX lists of cross-shard PRUNEs
    travel to the receivers' ranks (gsx_hb_px_*), which apply
    AcceptPXThreshold and pxConnect.  Counters summed over ranks and the PX
    connection records of all ranks == one engine; states equal too."""
    import heartbeat_cases as hc

    n, d, T, seed = 1500, 8, 2, 43
    ov = pc.overlay(n, d, seed, mix_protocols=True, direct_frac=0.02)
    gp = hc.be_default_params()
    gp.do_px = 1
    full = gsx.Engine(T)
    app = pc.setup(full, ov, T, seed, mesh_degree=10, disconnect_frac=0.05)
    full.set_gossipsub_params(gp)
    full.hb_set_px_log(1 << 20)
    st0 = full.export_state()
    E = ov.n_pairs
    rank_lo = synth.shard_ranges(n, world)
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        sh = synth.shard_of(ov, lo, hi)
        a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
        e = gsx.Engine(T)
        _params(e, T)
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.import_state(_slice_state(st0, T, E, a, b))
        e.set_app_scores(app[a:b])
        e.set_gossipsub_params(gp)
        e.hb_set_px_log(1 << 20)
        engines.append((e, a, b))
    runners = shard.run_local(world, "cuda:0", lambda tp, e: shard.RangeSharded(e, rank_lo, tp),
                              [(e,) for e, _, _ in engines])
    tot_px = tot_connect = cross = 0
    for k in range(3):
        tick, now = 60 + k, pc.T0 + (3 + k) * abi.SECOND
        want = full.heartbeat(tick, now, seed).as_dict()
        res = shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.heartbeat(tick, now, seed))[1],
                              [(r,) for r in runners])
        assert res[0][1] == want, (k, res[0][1], want)
        recs = np.concatenate([e.hb_px_records() for e, _, _ in engines])
        recs = recs[np.lexsort(recs.T[::-1])]
        assert np.array_equal(recs, full.hb_px_records()), k
        snap = hc.snapshot(full)
        for (e, a, b) in engines:
            got = hc.snapshot(e)
            for f in abi.STATE_FIELDS:
                assert np.array_equal(got[f].view(np.uint8), _slice_state(snap, T, E, a, b)[f].view(np.uint8)), (k, f)
            assert np.array_equal(np.asarray(got["backoff"]).reshape(-1), _slice_te(snap["backoff"], T, E, a, b)), k
        tot_px += want["px_prunes"]
        tot_connect += want["px_connect"]
        rk = np.searchsorted(rank_lo, recs[:, [0, 2]].astype(np.int64), side="right") - 1
        cross += int((rk[:, 0] != rk[:, 1]).sum())  # PX lists that travelled to another rank
    assert tot_px > 0 and tot_connect > 0 and cross > 0, (tot_px, tot_connect, cross)


def test_sharded_exchange_pending_refuses_other_calls(gpu_ok):
    """While a sharded gossip exchange is in flight (gsx_hb_end .. gsx_gx_end)
    a new round, a propagation, a state import / export or the backoff import
    is refused with GSX_ESTATE (the exchange holds the round's sets and the
    mcache Shift); the exchange then completes as usual."""
    import gossip_cases as gc

    n, d, seed, T, world = 600, 6, 53, 1, 2
    ov = pc.overlay(n, d, seed)
    full = gsx.Engine(T)
    app = pc.setup(full, ov, T, seed, mesh_degree=6)
    gp = gc.params()
    st0 = full.export_state()
    E = ov.n_pairs
    rank_lo = synth.shard_ranges(n, world)
    engines = []
    for k in range(world):
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        sh = synth.shard_of(ov, lo, hi)
        a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
        e = gsx.Engine(T)
        _params(e, T)
        e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.import_state(_slice_state(st0, T, E, a, b))
        e.set_app_scores(app[a:b])
        e.set_gossipsub_params(gp)
        engines.append(e)
    refused = []

    class Probe(shard.RangeSharded):
        def _gx_exchange(self, n_sets):
            be = self.be
            assert be.gx_pending() is not None
            for call in (lambda: be.hb_begin(9, pc.T0, 1), lambda: be.export_state(),
                         lambda: be.prop_begin(pc.messages(n, 4, 1), pc.config(abi.GSX_ROUTER_GOSSIPSUB)),
                         lambda: be.import_backoff(np.zeros((T, be.n_pairs), dtype=np.int64))):
                with pytest.raises(gsx.GsxError) as ex:
                    call()
                refused.append(ex.value.code == abi.GSX_ESTATE)
            return super()._gx_exchange(n_sets)

    runners = shard.run_local(world, "cuda:0", lambda tp, e: Probe(e, rank_lo, tp), [(e,) for e in engines])
    cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=0, max_hops=2, latency_ms=5, seed=seed)
    ms = pc.messages(n, 40, seed)
    shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.propagate(ms, cfg))[1],
                    [(r,) for r in runners])
    res = shard.run_local(world, "cuda:0",
                          lambda tp, r: (setattr(r, "tp", tp), r.heartbeat(1, pc.T0 + abi.SECOND, 5))[1],
                          [(r,) for r in runners])
    assert refused and all(refused), refused
    assert all(e.gx_pending() is None for e in engines)
    assert res[0][1]["iwant_msgs"] > 0
