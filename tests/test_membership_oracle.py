"""Topic membership in the CPU oracle: gs.p.topics filters
every peer choice, meshes exist only for joined topics, publishers that have
not joined use their fanout (gossipsub.go:981-998), which the heartbeat expires
after FanoutTTL and keeps at D (:1517-1554); Join / Leave (:1015-1082)."""
import numpy as np

import membership_cases as mc
import oracle as orc
from gsx import abi


def _pairs(ov):
    obs = np.repeat(np.arange(len(ov.row_ptr) - 1), np.diff(ov.row_ptr))
    return obs, np.asarray(ov.col)


def test_meshes_only_between_joined_nodes():
    """Meshes hold joined peers; a peer that leaves drops out of the meshes of
    its own mesh peers (its PRUNEs), but stays where the mesh was one-sided:
    unsubscription does not touch the router's mesh (pubsub.go handles it)."""
    be = orc.Oracle(2)
    ov, outs, snaps, mems, props = mc.membership_run(be, leave_at=6)
    obs, peer = _pairs(ov)
    for k, (st, (joined, fanout, lastpub)) in enumerate(zip(snaps, mems)):
        inm = (st["rec_flags"].reshape(2, -1) & abi.GSX_REC_IN_MESH) != 0
        for t in range(2):
            jt = (joined >> np.uint64(t)) & np.uint64(1)
            m = inm[t]
            assert np.all(jt[obs[m]] == 1), (k, t)  # gs.mesh[topic] exists only when joined
            if k < 6:
                assert np.all(jt[peer[m]] == 1), (k, t)


def test_unjoined_nodes_never_receive_and_sources_use_fanout():
    be = orc.Oracle(2)
    ov, outs, snaps, mems, props = mc.membership_run(be)
    obs, peer = _pairs(ov)
    used_fanout = 0
    for k, ((out, hop), (joined, fanout, lastpub)) in enumerate(zip(props, mems)):
        t = k % 2
        jt = ((joined >> np.uint64(t)) & np.uint64(1)).astype(bool)
        recv = (hop != 0xFF) & (hop != 0)
        assert not np.any(recv[:, ~jt])  # gs.p.topics: nobody sends to an unjoined node
        assert out["deliveries"] > 0
    j, f, lp = be.export_membership()
    # fanouts exist for unjoined publishers, hold <= D subscribed peers
    has = f != 0
    assert has.any()
    for t in range(2):
        ft = ((f >> np.uint64(t)) & np.uint64(1)).astype(bool)
        assert np.all(((j[peer[ft]] >> np.uint64(t)) & np.uint64(1)) == 1)
        assert np.all(((j[obs[ft]] >> np.uint64(t)) & np.uint64(1)) == 0)
        cnt = np.bincount(obs[ft], minlength=len(j))
        assert cnt.max() <= 6


def test_fanout_expires_after_ttl():
    be = orc.Oracle(2)
    mc.membership_run(be, ticks=8, fanout_ttl_s=1)
    _, f1, lp1 = be.export_membership()
    be2 = orc.Oracle(2)
    mc.membership_run(be2, ticks=8, fanout_ttl_s=100)
    _, f2, lp2 = be2.export_membership()
    assert np.count_nonzero(lp1) < np.count_nonzero(lp2)


def test_join_grafts_and_leave_prunes():
    be = orc.Oracle(2)
    ov, outs, snaps, mems, props = mc.membership_run(be)
    j = dict((k, o) for k, o in outs if k != "hb")
    assert j["join"]["grafts"] > 0 and j["join"]["graft_accepted"] + j["join"]["graft_rejected"] > 0
    assert j["leave"]["prunes"] > 0 and j["leave"]["prunes_handled"] > 0
