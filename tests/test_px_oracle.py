"""Peer exchange on PRUNE in the oracle (gossipsub.go:811-843, 861-910,
1814-1850), checked against what the reference code decides: the PX list is
getPeers(topic, PrunePeers, xp != p && score >= 0), it is left out for peers
without feature PX and for negative-score prunes, a receiver below
AcceptPXThreshold ignores it, and pxConnect only queues peers the receiver is
not connected to.  Parity unpinned by reference fixtures (the reference's PX
test, TestGossipsubPeerExchange, is a timing-based network run)."""
import numpy as np

import heartbeat_cases as hc
import oracle as orc
import px_cases as xc
from gsx import abi


def test_star_prune_lists_every_other_peer():
    out, rec, pair = xc.star_case(orc.Oracle(1))
    assert out["prunes"] == 8  # 14 mesh peers > Dhi = 12: pruned down to D = 6
    assert out["px_prunes"] == 8 and out["px_peers"] == 8 * 13
    assert out["px_connect"] == 8 * 13 and out["px_ignored"] == 0
    assert len(rec) == 104
    recv = sorted(set(rec[:, 0].tolist()))
    assert len(recv) == 8
    for r in recv:
        mine = rec[rec[:, 0] == r]
        assert sorted(mine[:, 1].tolist()) == [k for k in range(1, 15) if k != r]  # every other leaf
        assert (mine[:, 2] == 0).all() and (mine[:, 3] == 0).all()  # pruner 0, topic 0, kind 0


def test_star_prune_peers_truncates():
    out, rec, _ = xc.star_case(orc.Oracle(1), prune_peers=5)
    assert out["px_peers"] == 8 * 5 and out["px_connect"] == 8 * 5
    for r in set(rec[:, 0].tolist()):
        assert (rec[:, 0] == r).sum() == 5


def test_star_receiver_below_accept_threshold_ignores():
    out, rec, _ = xc.star_case(orc.Oracle(1), leaf_view=-1.0)  # below AcceptPXThreshold 0, above graylist
    assert out["px_prunes"] == 8 and out["px_ignored"] == 8
    assert out["px_connect"] == 0 and len(rec) == 0


def test_star_no_px_feature_sends_no_list():
    out, rec, _ = xc.star_case(orc.Oracle(1), no_px=True)
    assert out["prunes"] == 8 and out["px_prunes"] == 0 and len(rec) == 0


def test_star_negative_score_prune_without_px():
    # leaves 1 and 2 score -5 at the hub: pruned first, without PX (:1361-1368),
    # and never listed to anyone (score(xp) >= 0)
    out, rec, _ = xc.star_case(orc.Oracle(1), n_leaves=16, hub_view={1: -5.0, 2: -5.0})
    assert out["prunes"] == 10  # 2 negative, then 14 -> 6
    assert out["px_prunes"] == 8
    assert not np.isin(rec[:, 0], [1, 2]).any()
    assert not np.isin(rec[:, 1], [1, 2]).any()
    assert out["px_peers"] == 8 * 13


def test_px_off_by_default():
    o = orc.Oracle(1)
    _, outs, _ = hc.mesh_run(o, 300, 6, 1, seed=5, ticks=3, mesh_degree=14)
    assert all(x["px_prunes"] == x["px_peers"] == x["px_connect"] == x["px_ignored"] == 0 for x in outs)


def test_px_run_invariants():
    o = orc.Oracle(2)
    ov, outs, recs, _ = xc.px_run(o, 400, 8, 2, seed=11, ticks=3, prune_peers=4, join_frac=0.85, mesh_degree=3,
                                  d_hi=6, accept_px=1.0)
    rows = {u: set(ov.col[ov.row_ptr[u]:ov.row_ptr[u + 1]].tolist()) for u in range(ov.n)}
    st = o.export_state()
    conn = (st["pair_flags"] & abi.GSX_PAIR_CONNECTED) != 0
    tot = {k: sum(x[k] for x in outs) for k in ("px_prunes", "px_peers", "px_connect", "px_ignored", "prunes")}
    assert tot["px_prunes"] > 0 and tot["px_connect"] > 0 and tot["px_ignored"] > 0
    assert tot["px_peers"] <= 4 * tot["px_prunes"]
    kinds = np.concatenate([r[:, 3] >> 8 for r in recs])
    assert (kinds == 0).any() and (kinds == 1).any()  # (A) PRUNEs and (B) answers both carry PX
    for out, rec in zip(outs, recs):
        assert len(rec) == out["px_connect"]
        for recv, cand, pruner, tk in rec.tolist():
            assert cand != recv and pruner in rows[recv] and cand in rows[pruner]
            if cand in rows[recv]:  # a known peer is a candidate only while disconnected
                q = ov.row_ptr[recv] + int(np.searchsorted(ov.col[ov.row_ptr[recv]:ov.row_ptr[recv + 1]], cand))
                assert not conn[q]
        # at most PrunePeers candidates per PRUNE
        if len(rec):
            _, cnt = np.unique(rec[:, [0, 2, 3]], axis=0, return_counts=True)
            assert cnt.max() <= 4


def test_px_leave_and_join_rounds():
    res = xc.px_member_run(orc.Oracle(2))
    (hb, _), (lv, lrec), (jn, jrec) = res
    assert lv["prunes"] > 0 and lv["px_prunes"] > 0 and lv["px_connect"] == len(lrec)
    assert (lrec[:, 3] >> 8 == 0).all() and (lrec[:, 3] & 0xFF == 0).all()  # Leave PRUNEs of topic 0
    assert jn["px_connect"] == len(jrec)
