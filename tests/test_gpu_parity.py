"""Parity of the HIP engine (through the C ABI) with the CPU oracle and the
reference's known answers.  Bit-exact: scores are FP64 computed with the same
operations in the same order (-ffp-contract=off on both sides), counters are
exact, flags/times are integers."""
import numpy as np
import pytest

import gsx
import oracle as orc
import randomized as R
from gsx import abi, synth
from scenario import load_json, run_scenario

pytestmark = pytest.mark.gpu

KAT = load_json("score_kat.json")


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def assert_same_state(got, want, where=""):
    for f in abi.STATE_FIELDS:
        g, w = got[f], want[f]
        if not np.array_equal(bits(g), bits(w)):
            bad = np.nonzero(bits(g).reshape(len(g), -1).any(1) != bits(w).reshape(len(w), -1).any(1))[0]
            idx = np.nonzero(g != w)[0][:5]
            raise AssertionError(f"{where} field {f}: {np.count_nonzero(g != w)} differ, e.g. {idx} {g[idx]} vs {w[idx]}")


def assert_same_scores(got, want, where=""):
    if not np.array_equal(got.view(np.uint64), want.view(np.uint64)):
        idx = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0][:8]
        raise AssertionError(f"{where}: {len(np.nonzero(got != want)[0])} scores differ, e.g. {idx}: {got[idx]} vs {want[idx]}")


@pytest.mark.parametrize("sc", KAT, ids=[s["name"] for s in KAT])
def test_engine_score_kat(gpu_ok, sc):
    bad = run_scenario(sc, lambda T: gsx.Engine(T))
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("seed,n,d,T", [(1, 64, 2, 2), (7, 300, 3, 3), (11, 1500, 6, 4), (23, 800, 4, 9)])
def test_engine_matches_oracle_random_calls(gpu_ok, seed, n, d, T):
    ov = R.small_overlay(n, d, seed, max(8, n // 6))
    ops = R.make_ops(ov, T, seed, n_steps=300)
    got = R.replay(gsx.Engine(T), ov, T, ops)
    want = R.replay(orc.Oracle(T), ov, T, ops)
    assert len(got) == len(want)
    for i, ((gs, gst, gn), (ws, wst, wn)) in enumerate(zip(got, want)):
        assert gn == wn, f"check {i}: delivery records {gn} vs {wn}"
        assert_same_scores(gs, ws, f"check {i}")
        assert_same_state(gst, wst, f"check {i}")


@pytest.mark.parametrize("seed,n,d,T", [(3, 200, 3, 3), (5, 3000, 6, 2), (9, 9000, 4, 2)])
def test_engine_score_calls_interleaved(gpu_ok, seed, n, d, T):
    """Score() after every single event / tracer call (incremental re-scoring of
    the flushed observers' rows, the host score copy of small engines, and the
    full re-score of engines above it) == the oracle's score() at the same point."""
    ov = R.small_overlay(n, d, seed, max(8, n // 6))
    ops = R.make_ops(ov, T, seed, n_steps=120)
    got = R.interleaved_score_calls(gsx.Engine(T), ov, T, ops, seed)
    want = R.interleaved_score_calls(orc.Oracle(T), ov, T, ops, seed)
    assert len(got) == len(want) > 100
    assert_same_scores(got, want, "interleaved Score()")


@pytest.mark.parametrize("seed,n,d,T", [(4, 200, 3, 3), (6, 3000, 6, 2), (11, 16000, 6, 2)])
def test_engine_score_many_interleaved(gpu_ok, seed, n, d, T):
    """gsx_score_many (one RPC's gates and Publish targets at once) after
    every single event / tracer call: the one-launch drop-in round trip
    (k_dropin: events, the touched rows re-scored into the host-mapped copy)
    on small engines, the gather on the 16000-node one (above the host-copy
    size) == the oracle's score() of the same pairs."""
    ov = R.small_overlay(n, d, seed, max(8, n // 6))
    ops = R.make_ops(ov, T, seed, n_steps=120)
    got = R.interleaved_score_calls(gsx.Engine(T), ov, T, ops, seed, per_call=6, many=True)
    want = R.interleaved_score_calls(orc.Oracle(T), ov, T, ops, seed, per_call=6, many=True)
    assert len(got) == len(want) > 100
    assert_same_scores(np.array(got), np.array(want), "interleaved score_many")


@pytest.mark.parametrize("n,T,p_disc,p_abs", [(20000, 8, 0.0, 0.0), (30000, 8, 0.1, 0.05), (40000, 1, 0.05, 0.05),
                                              (5000, 5, 0.2, 0.2)])
def test_engine_refresh_matches_oracle_synthetic(gpu_ok, n, T, p_disc, p_abs):
    """cfg3-style synthetic state: several refresh+score passes."""
    ov = synth.connect_some_overlay(n, d=6, sybil_frac=0.2, sybils_per_ip=50)
    now = R.T0
    st = synth.synthetic_state(ov, T, now, p_disconnected=p_disc, p_absent=p_abs)
    pp = synth.bench_peer_params()
    tp = synth.spam_test_topic_params()
    app = synth.uniform(synth.SEED, synth.TAG_STATE, np.arange(ov.n_pairs, dtype=np.uint64), 11) * 4 - 2
    bes = []
    for be in (gsx.Engine(T), orc.Oracle(T)):
        be.set_peer_params(pp)
        for t in range(T):
            be.set_topic_params(t, tp)
        be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
        be.import_state(st)
        be.set_app_scores(app)
        bes.append(be)
    eng, ora = bes
    assert_same_scores(eng.scores(), ora.scores(), "before refresh")
    for k in range(4):
        now += abi.SECOND
        eng.refresh(now)
        ora.refresh(now)
        assert_same_scores(eng.scores(), ora.scores(), f"refresh {k}")
    assert_same_state(eng.export_state(), ora.export_state(), "final")


def test_engine_scores_full_size_properties(gpu_ok):
    """At the bench size (1M peers x 8 topics) compare a contiguous sample of
    pairs with the oracle run on the same sample, and check refresh is the
    same function of its inputs when replayed (import -> refresh twice)."""
    n, T = 1_000_000, 8
    ov = synth.connect_some_overlay(n, d=6)
    now = R.T0
    st = synth.synthetic_state(ov, T, now, p_disconnected=0.02)
    pp = synth.bench_peer_params()
    tp = synth.spam_test_topic_params()
    eng = gsx.Engine(T)
    eng.set_peer_params(pp)
    for t in range(T):
        eng.set_topic_params(t, tp)
    eng.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    eng.import_state(st)
    eng.refresh(now + abi.SECOND)
    s1 = eng.scores()
    eng.import_state(st)
    eng.refresh(now + abi.SECOND)
    s2 = eng.scores()
    assert_same_scores(s1, s2, "replay")
    # oracle on a sample: observers [0, 2000) -> their pairs
    n_obs = 2000
    p1 = int(ov.row_ptr[n_obs])
    sub_rp = ov.row_ptr[: n_obs + 1]
    # the sample keeps the full node id space so IPs/cols are unchanged
    ora = orc.Oracle(T)
    ora.set_peer_params(pp)
    for t in range(T):
        ora.set_topic_params(t, tp)
    rp = np.concatenate([sub_rp, np.full(n - n_obs, p1, dtype=np.int64)])
    ora.load_overlay(rp, ov.col[:p1], None, ov.node_ips)
    E = ov.n_pairs
    sub = {f: (st[f].reshape(T, E)[:, :p1].reshape(-1) if f in abi.RECORD_FIELDS else st[f][:p1]) for f in abi.STATE_FIELDS}
    ora.import_state(sub)
    ora.set_app_scores(np.zeros(p1))
    ora.refresh(now + abi.SECOND)
    assert_same_scores(s1[:p1], ora.scores(), "sample")


def test_engine_set_pair_ips_matches_oracle(gpu_ok):
    """gsx_set_pair_ips (refreshIPs / setIPs) == the oracle, step by step."""
    import ip_cases as ic

    got, _ = ic.run(gsx.Engine(1))
    want, _ = ic.run(orc.Oracle(1))
    for i, (g, w) in enumerate(zip(got, want)):
        assert_same_scores(g, w, f"step {i}")


@pytest.mark.parametrize("seed", [4, 12])
def test_engine_snapshot_matches_oracle(gpu_ok, seed):
    """gsx_peer_score_snapshot (inspectScoresExtended, score.go:463-493) == the
    oracle's PeerScoreSnapshot fields after a random call sequence (IP moves,
    retention, grafts, deliveries)."""
    T = 3
    ov = R.small_overlay(900, 4, seed, 150)
    ops = R.make_ops(ov, T, seed, n_steps=150)
    g, w = gsx.Engine(T), orc.Oracle(T)
    R.replay(g, ov, T, ops)
    R.replay(w, ov, T, ops)
    gs, ws = g.snapshot(), w.snapshot()
    assert int(gs["present"].sum()) > 0
    for f in ws:
        assert np.array_equal(np.asarray(gs[f]).view(np.uint8), np.asarray(ws[f]).view(np.uint8)), f
