"""The gossip exchange on the GPU vs the CPU oracle (gsx.h heartbeat step (D):
handleIHave / handleIWant, gossipsub.go:615-716; promises and their P7
penalty, gossip_tracer.go:48-153, gossipsub.go:1578-1583): every round's
counters, records, scores (P7 through behaviourPenalty), IHAVEs and every
node's cached ids (the recovered copies) are equal."""
import numpy as np
import pytest

import gossip_cases as gc
import gsx
import oracle as orc
import promise_cases as pc
from gsx import abi

pytestmark = pytest.mark.gpu

FIELDS = list(abi.STATE_FIELDS) + ["backoff", "scores", "ihave_len", "ihave_digest"]


def _same(g, w):
    ov, go, gs, gcache = g
    _, wo, ws, wcache = w
    for k in range(len(go)):  # the first tick that differs: its counters, then its state
        diff = {x: (go[k][x], wo[k][x]) for x in go[k] if go[k][x] != wo[k][x]}
        assert not diff, f"tick {k}: {diff}"
        for f in FIELDS:
            a, b = np.asarray(gs[k][f]), np.asarray(ws[k][f])
            if not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                bad = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
                pytest.fail(f"tick {k} field {f}: {len(bad)} differ, first {bad[:5].tolist()} "
                            f"gpu {a.reshape(-1)[bad[:5]].tolist()} oracle {b.reshape(-1)[bad[:5]].tolist()}")
    for v, (a, b) in enumerate(zip(gcache, wcache)):
        assert sorted(a.tolist()) == sorted(b.tolist()), v


@pytest.mark.parametrize("kw", [
    dict(),                                   # HistoryGossip == HistoryLength (reference default)
    dict(history_gossip=3),                   # everything asked is served
    dict(exchange_from=5, ticks=10),          # unanswered IHAVEs: broken promises, P7
    dict(invalid=0.3, ticks=6),               # recovered invalid messages: P4
    dict(T=1, n=500, d=8, msgs=70, ticks=6),  # two words per batch
    dict(max_ihave_length=9, ticks=6),        # every list truncated per target (Floyd subsets)
    dict(max_ihave_length=40, msgs=30, ticks=8, invalid=0.2),  # lists cross MaxIHaveLength as the window fills
    dict(prefill=3, ticks=6, exchange_from=2),  # 3 of 4 promise slots taken: the exchange's promises grow them
    dict(T=1, n=300, msgs=4200, hops=2, ticks=4),  # 66-word sets: no common words, every asker heavy (k_gx_node)
    dict(T=1, n=10, d=3, msgs=6, hops=1, ticks=6),  # 10 nodes: a one-node frontier is already a dense hop
    dict(max_ihave_messages=0, ticks=4),      # MaxIHaveMessages 0: every IHAVE RPC ignored (peerhave limit)
    # batches that reach most nodes: most receivers miss a few messages (<= GX_POOR, k_gx_ask filters
    # their senders by the common2 words), a few miss many (unfiltered)
    dict(hops=5, msgs=40, ticks=6),
    dict(T=1, n=400, d=8, hops=4, msgs=100, ticks=6, invalid=0.1),
], ids=["default", "hg3", "broken", "invalid", "two_words", "trunc9", "trunc40", "prefill", "wide", "tiny10",
        "no_ihave_msgs", "reach5", "reach4_two_words"])
def test_gossip_exchange_matches_oracle(gpu_ok, kw):
    T = kw.get("T", 2)
    g = gc.exchange_run(gsx.Engine(T), **kw)
    w = gc.exchange_run(orc.Oracle(T), **kw)
    _same(g, w)
    if kw.get("max_ihave_messages", 1) == 0:
        assert sum(o["iwant_msgs"] for o in g[1]) == 0 and sum(o["ihave_ignored"] for o in g[1]) > 0
    else:
        assert sum(o["iwant_msgs"] for o in g[1]) > 0


# Heartbeats every second, batches 100 ms after one with 5 ms hops: an old
# copy's validation time is the batch's now + 5 ms x its arrival hop, or the
# heartbeat that recovered it.  892 ms: the window boundary falls between hops
# 1 and 2 of the last batch (hop 2 inside, hops 0 and 1 outside); 897 ms:
# between the source and hop 1; 1000 ms: the copies recovered one heartbeat
# earlier are inside too; 2500 ms: two heartbeats back, older ones outside;
# 2 ms hops + 1 ms validation delay with the boundary between hops 2 and 3.
WINDOW_CASES = [
    dict(window_ms=892, hops=3),
    dict(window_ms=897, hops=3),
    dict(window_ms=1000, hops=3, history_gossip=3),
    dict(window_ms=2500, hops=2, ticks=6),
    dict(window_ms=893.5, hops=4, latency_ms=2, delay_ms=1.0, T=1, msgs=40),
]


@pytest.mark.parametrize("kw", WINDOW_CASES, ids=["hop1_2", "src_hop1", "one_round", "two_rounds", "delay"])
def test_gossip_exchange_per_node_validation_time(gpu_ok, kw):
    """A forwarded duplicate counts for P3 iff now - the receiver's own
    validation time <= MeshMessageDeliveriesWindow (score.go:944-974: per
    (observer, message) drec.validated), with the window boundary between
    arrival hops / recovery rounds: engine == oracle."""
    T = kw.get("T", 2)
    g = gc.exchange_run(gsx.Engine(T), **kw)
    w = gc.exchange_run(orc.Oracle(T), **kw)
    _same(g, w)
    assert sum(o["fwd_duplicates"] for o in g[1]) > 0


def test_sets_cached_with_exchange_off_refuse_a_split_window(gpu_ok):
    """A batch propagated with the gossip exchange off keeps no arrival hops
    (its per-node validation times are not built): once the exchange is on, a
    heartbeat whose P3 window would split that set's copies is refused
    (GSX_ESTATE) rather than credited inexactly; a window that leaves them all
    on one side runs."""
    import heartbeat_cases as hc
    import propagation_cases as pcs

    for win, ok in ((892, False), (25, True)):
        e = gsx.Engine(1)
        ov = pcs.overlay(300, 6, 5)
        pcs.setup(e, ov, 1, 5, mesh_degree=6)
        from gsx import synth

        tp = synth.spam_test_topic_params()
        tp.mesh_message_deliveries_window_ns = int(win * abi.MILLISECOND)
        e.set_topic_params(0, tp)
        e.set_gossipsub_params(gc.params(gossip_exchange=0))
        now = hc.T0 + 3 * abi.SECOND
        cfg = pcs.config(abi.GSX_ROUTER_GOSSIPSUB, max_hops=3, latency_ms=5, seed=9)
        cfg.now_ns = now + 100 * abi.MILLISECOND
        e.propagate(pcs.messages(300, 24, 9), cfg)
        e.set_gossipsub_params(gc.params())
        if ok:
            e.heartbeat(1, now + abi.SECOND, 7)
        else:
            with pytest.raises(abi.GsxError):
                e.heartbeat(1, now + abi.SECOND, 7)


@pytest.mark.timeout(600)
def test_gossip_exchange_1024_per_heartbeat(gpu_ok):
    """1024 messages between heartbeats: the five-window gossip list holds up
    to 5,120 ids > MaxIHaveLength 5,000, so lists are truncated per target and
    the receivers ask from their subsets (done criterion of f1)."""
    kw = dict(T=1, n=2000, d=8, msgs=1300, hops=4, ticks=7)
    g = gc.exchange_run(gsx.Engine(1), **kw)
    w = gc.exchange_run(orc.Oracle(1), **kw)
    _same(g, w)
    outs = g[1]
    assert (g[2][-1]["ihave_len"] == 5000).sum() > 1000  # truncated lists went out (the snapshot of the last round)
    assert outs[-1]["iwant_msgs"] > 0 and outs[-1]["gossip_delivered"] > 0


@pytest.mark.parametrize("case", pc.load(), ids=lambda c: c["name"])
def test_promise_kat_gpu(gpu_ok, case):
    """gossip_tracer_test.go:12-97 through gsx_promise_* (tests/golden/promise_kat.json)."""
    assert pc.run(gsx.Engine(1), case) == []


def test_promise_slots_grow_gpu(gpu_ok):
    """1000 promises on one pair (AddPromise never refuses): the engine's per-pair
    slots double on demand; counts and GetBrokenPromises equal the oracle's."""
    from gsx import synth

    res = []
    for be in (gsx.Engine(1), orc.Oracle(1)):
        row_ptr, col = pc.star(3)
        be.set_peer_params(synth.bench_peer_params())
        be.load_overlay(row_ptr, col)
        for k in range(1000):
            be.promise_add(k % 2, [k, k + 1, k + 2], pc.T0 + k, seed=k)
        with pytest.raises(Exception):  # expiry 0: the free-slot mark, refused by both (gsx.h)
            be.promise_add(0, [7], 0)
        a = be.promise_count()
        cnt, tot = be.promise_broken(pc.T0 + 500)
        for k in range(0, 1000, 7):
            be.promise_fulfill(0, k)
        be.promise_throttle(1)
        res.append((a, cnt.tolist(), tot, be.promise_count()))
    assert res[0] == res[1]
