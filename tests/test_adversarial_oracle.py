"""cfg5 (sybil IP groups + invalid-message spam) on the CPU oracle: the
colocated sybils and the spammers score below the graylist threshold, and
one heartbeat takes every negative-score peer out of every mesh
(gossipsub.go:1351-1363)."""
import numpy as np

import adversarial_cases as ac
import oracle as orc
from gsx import abi


def test_sybils_are_graylisted_and_pruned():
    o = orc.Oracle(1)
    ov = ac.setup(o, 2500)
    sc = o.scores()
    syb = ac.sybil_pairs(ov)
    vic = ac.victim_pairs(ov)
    st = o.export_state()
    imd = st["invalid_message_deliveries"]
    assert vic.sum() > 0 and syb.sum() > 0
    # every colocated sybil seen by a victim: P6 = (50 - 1)^2 * -10 alone
    assert (sc[vic & syb] < ac.TH.graylist_threshold).all()
    # spammers with a non-trivial invalid count are graylisted everywhere:
    # P4 = imd^2 * -99 * TopicWeight 0.25 outweighs any capped positive part
    spam = syb & (imd > 10.0)
    assert spam.sum() > 0 and (sc[spam] < ac.TH.graylist_threshold).all()
    # honest peers: only the synthetic P3 deficits / P7 of cfg3's
    # initialisation can push a few of them down
    assert (sc[~syb] > ac.TH.graylist_threshold).mean() > 0.9
    assert np.median(sc[~syb]) > 0 > np.median(sc[syb])
    o.heartbeat(1, ac.T0 + 2 * abi.SECOND, 9)
    st = o.export_state()
    sc = o.scores()
    in_mesh = (st["rec_flags"] & abi.GSX_REC_IN_MESH) != 0
    assert not (in_mesh & (sc < 0)).any()
    assert in_mesh.sum() > 0
