"""The oracle's heartbeat (gossipsub.go:1303-1604, 718-859) against the
reference's own heartbeat assertions, restated for the synchronous-round
contract of gsx.h.  Parity of the heartbeat is unpinned by golden vectors (the
reference tests are timing-based network runs); these checks pin
the oracle to the behaviour those tests assert."""
import numpy as np
import pytest

import heartbeat_cases as hc
import oracle as orc
from gsx import abi

S = abi.SECOND
MS = abi.MILLISECOND


def test_default_params_match_reference():
    gp = orc.default_gossipsub_params()  # DefaultGossipSubParams, gossipsub.go:230-260
    assert (gp.d, gp.d_lo, gp.d_hi, gp.d_score, gp.d_out) == (6, 5, 12, 4, 2)
    assert (gp.opportunistic_graft_peers, gp.opportunistic_graft_ticks) == (2, 60)
    assert gp.prune_backoff_ns == 60 * S and gp.graft_flood_threshold_ns == 10 * S
    assert (gp.d_lazy, gp.history_length, gp.history_gossip, gp.max_ihave_length) == (6, 5, 5, 5000)
    assert gp.gossip_factor == 0.25


def test_opportunistic_grafting():
    o = orc.Oracle(1)
    out, pair = hc.opportunistic_graft_case(o)
    out = out.as_dict()
    assert out["grafts"] == 2 and out["graft_accepted"] == 2
    assert out["prunes"] == 0 and out["graft_rejected"] == 0
    st = o.export_state()
    mesh = st["rec_flags"] & abi.GSX_REC_IN_MESH
    node0 = [k for k in range(1, 11) if mesh[pair[(0, k)]]]
    assert node0[:6] == [1, 2, 3, 4, 5, 6] and len(node0) == 8
    assert all(k >= 7 for k in node0[6:])
    # the chosen peers accepted: their side of the link is in the mesh too
    assert all(mesh[pair[(k, 0)]] for k in node0)
    assert out["mesh_links"] == 8 + 6 + 2


def test_opportunistic_grafting_only_on_its_ticks():
    o = orc.Oracle(1)
    hc.opportunistic_graft_case(o)
    out = o.heartbeat(61, hc.T0 + 3 * S, 1234).as_dict()
    assert out["grafts"] == 0


def test_graft_during_backoff_is_penalised():
    rounds, pair = hc.graft_flood_case(orc.Oracle(1))
    pen = [r[0]["penalties"] for r in rounds]
    rej = [r[0]["graft_rejected"] for r in rounds]
    scores = [r[1] for r in rounds]
    # after the flood cutoff: 1 penalty; before it: 2 (gossipsub.go:752-770)
    assert pen == [1, 2, 2, 0]
    assert rej == [1, 1, 1, 0]  # a PRUNE answers every GRAFT until the attacker is graylisted
    assert scores[:3] == [-100.0, -900.0, -2500.0]  # -100 * bp^2
    assert scores[2] < -1000  # below the graylist threshold: the 4th GRAFT is ignored (AcceptFrom)
    assert rounds[3][0]["prunes_handled"] == 0
    # the attacker handled each PRUNE: backoff 200 ms (PRUNE carries 0 whole seconds, :825-830)
    t1 = hc.T0 + S
    a_to_l, l_to_a = pair[(1, 0)], pair[(0, 1)]
    assert rounds[0][2][0, a_to_l] == t1 + 200 * MS
    assert rounds[0][2][0, l_to_a] == t1 + 200 * MS
    assert rounds[2][2][0, l_to_a] == t1 + 40 * MS + 200 * MS


@pytest.mark.parametrize("mesh_degree,d", [(2, 6), (14, 9)], ids=["graft-up", "prune-down"])
def test_mesh_invariants(mesh_degree, d):
    n, T = 400, 2
    o = orc.Oracle(T)
    gp = orc.default_gossipsub_params()
    ov, outs, snaps = hc.mesh_run(o, n, d, T, seed=3, ticks=5, mesh_degree=mesh_degree, direct=0.02,
                                  gp=gp, first_tick=13, mostly_positive=True)
    E = ov.n_pairs
    ef = ov.edge_flags
    obs = ov.pair_observer()
    prev_mesh = None
    prev_backoff = np.zeros((T, E), dtype=np.int64)
    for k, (out, st) in enumerate(zip(outs, snaps)):
        now = hc.T0 + (3 + k) * S
        present = (st["pair_flags"] & abi.GSX_PAIR_PRESENT) != 0
        mesh = ((st["rec_flags"].reshape(T, E) & abi.GSX_REC_IN_MESH) != 0) & present
        assert out["mesh_links"] == int(mesh.sum())
        # negative-score peers are never left in (or taken into) a mesh;
        # setup() gave 8 % of the pairs app score -500
        assert not (mesh & (st["scores"] < -400)[None, :]).any()
        if prev_mesh is not None:
            left = prev_mesh & ~mesh
            joined = mesh & ~prev_mesh
            assert (st["backoff"][left] >= now + gp.prune_backoff_ns).all()
            assert ((prev_backoff[joined] == 0) | (prev_backoff[joined] <= now)).all()
            assert not (joined & ((ef & abi.GSX_EDGE_DIRECT) != 0)).any()
        # mesh sizes: the heartbeat keeps them in [Dlo, Dhi] for nodes with
        # enough eligible candidates (the reference's mesh-size tests)
        deg = np.zeros((T, n), dtype=np.int64)
        for t in range(T):
            np.add.at(deg[t], obs[mesh[t]], 1)
        assert (deg <= gp.d_hi + 3).all()  # receivers take outbound GRAFTs above Dhi (:791-797)
        if k >= 1 and mesh_degree < gp.d_lo:  # graft-up fills the meshes
            assert np.median(deg) >= gp.d_lo
        if mesh_degree > gp.d_hi:  # prune-down: PRUNEs cross in one round, backoff blocks regrafts
            assert np.median(deg) <= gp.d
        prev_mesh = mesh
        prev_backoff = st["backoff"]
    assert sum(o["grafts"] for o in outs) > 0
    assert outs[2]["backoff_cleared"] >= 0  # tick 15 ran clearBackoff
    if mesh_degree > gp.d_hi:
        assert outs[0]["prunes"] > 0


def test_clear_backoff_runs_every_15_ticks():
    o = orc.Oracle(1)
    hc.opportunistic_graft_case(o)
    b = o.export_backoff()
    b[0, :] = hc.T0  # long expired
    o.import_backoff(b)
    assert o.heartbeat(14, hc.T0 + 10 * S, 1).as_dict()["backoff_cleared"] == 0
    out = o.heartbeat(15, hc.T0 + 10 * S, 1).as_dict()
    assert out["backoff_cleared"] == b.size
    # expiry + 2 heartbeat intervals of slack (gossipsub.go:1596)
    b[0, :] = hc.T0 + 9 * S
    o.import_backoff(b)
    assert o.heartbeat(30, hc.T0 + 10 * S, 1).as_dict()["backoff_cleared"] == 0


def test_heartbeat_is_deterministic_in_its_seed():
    snaps = []
    for seed in (5, 5, 6):
        o = orc.Oracle(1)
        ov = hc.pc.overlay(300, 8, 11)
        hc.pc.setup(o, ov, 1, 11, mesh_degree=14)
        o.heartbeat(1, hc.T0 + 3 * S, seed)
        snaps.append(o.export_state()["rec_flags"])
    assert np.array_equal(snaps[0], snaps[1])
    assert not np.array_equal(snaps[0], snaps[2])


def _check_message_cache(v):
    ids = lambda a, b: list(range(a, b))  # noqa: E731
    assert list(v["first"]) == ids(0, 10)
    assert list(v["second"]) == ids(10, 20) + ids(0, 10)  # newest window first
    assert sorted(v["second_all"]) == ids(0, 20)
    assert sorted(v["cache"]) == ids(10, 60)  # 50 messages, the first window shifted out
    assert list(v["gossip"]) == ids(50, 60) + ids(40, 50) + ids(30, 40)
    assert list(v["receiver"]) == list(v["gossip"])


def test_message_cache_windows():
    _check_message_cache(hc.message_cache_case(orc.Oracle(1)))


def test_gossip_emission():
    """TestGossipsubGossip (gossipsub_test.go:338-383): messages reach non-mesh
    peers through IHAVE.  Every IHAVE goes to a non-mesh, non-direct peer,
    carries all of the sender's gossip-window ids, and each sender picks
    max(Dlazy, GossipFactor * eligible) of its eligible peers."""
    n, T = 400, 1
    o = orc.Oracle(T)
    ov, outs, snaps = hc.mesh_run(o, n, 9, T, seed=8, ticks=2, mesh_degree=4, prop_msgs=40, mostly_positive=True)
    gp = orc.default_gossipsub_params()
    out, st = outs[1], snaps[1]  # the second heartbeat sees the first batch in its cache
    ln, dg = st["ihave_len"][0], st["ihave_digest"][0]
    sent = ln > 0
    assert out["ihave_msgs"] == int(sent.sum()) > 0
    assert out["ihave_ids"] == int(ln.sum())
    E = ov.n_pairs
    mesh = (st["rec_flags"][:E] & abi.GSX_REC_IN_MESH) != 0
    was = (snaps[0]["rec_flags"][:E] & abi.GSX_REC_IN_MESH) != 0
    assert not (sent & mesh & was).any()  # in the mesh all through the maintenance: pushed to, not gossiped
    assert not (sent & ((ov.edge_flags & abi.GSX_EDGE_DIRECT) != 0)).any()
    obs = ov.pair_observer()
    for v in range(0, n, 37):
        row = np.arange(ov.row_ptr[v], ov.row_ptr[v + 1])
        L = len(o.mcache_ids(v, 0, gp.history_gossip))
        # the heartbeat Shifted after emitting: the emitted window is now windows 1..
        assert (ln[row][sent[row]] <= L + 0).all()
        k = int(sent[row].sum())
        assert k <= max(gp.d_lazy, len(row))
    assert (obs[sent] >= 0).all()


def test_gossip_truncates_per_peer():
    gp = orc.default_gossipsub_params()
    gp.max_ihave_length = 7
    o = orc.Oracle(1)
    ov, outs, snaps = hc.mesh_run(o, 300, 9, 1, seed=4, ticks=2, mesh_degree=4, prop_msgs=50, gp=gp,
                                  mostly_positive=True)
    ln, dg = snaps[1]["ihave_len"][0], snaps[1]["ihave_digest"][0]
    assert set(np.unique(ln[ln > 0])) == {7}
    # each target gets its own reshuffled subset (gossipsub.go:1708-1716)
    for v in range(300):
        row = np.arange(ov.row_ptr[v], ov.row_ptr[v + 1])
        d = dg[row][ln[row] > 0]
        if len(d) >= 2:
            assert len(set(d.tolist())) > 1
            break
    else:
        raise AssertionError("no node gossiped to two peers")
