"""gsx_set_pair_ips semantics on the oracle (setIPs, score.go:1021-1059):
P6 follows the peers' current IP lists; absent peers are counted from their
next AddPeer; a peer's list is a set (a duplicated IP counts it once but is
penalised twice, score.go:373-377)."""
import numpy as np

import ip_cases as ic
import oracle as orc


def test_set_pair_ips_moves_p6():
    out, K = ic.run(orc.Oracle(1))
    np.testing.assert_array_equal(out[0], [0, -4, -4, -4, 0])
    np.testing.assert_array_equal(out[1], [-1, -1, -1, -1, 0])
    np.testing.assert_array_equal(out[2], out[1])
    # 1 -> {A, D}, 2 -> {B, C, E}; E holds 2 twice
    np.testing.assert_array_equal(out[3], [-1, -4, -4, -1, -8])
    # B alone on 7, C without addresses, 2 -> {E}
    np.testing.assert_array_equal(out[4], [-1, 0, 0, -1, 0])
    # retained A leaves 1 for 3: {A} (E's 3 was never E's), D alone on 1
    np.testing.assert_array_equal(out[5], [0, 0, 0, 0, 0])


def test_oracle_snapshot_ip_factor():
    """PeerScoreSnapshot.IPColocationFactor is the unweighted P6 (weight -1 here: -score)."""
    o = orc.Oracle(1)
    out, K = ic.run(o)
    snap = o.snapshot()
    np.testing.assert_array_equal(snap["ip_colocation_factor"], -out[-1] + 0.0)
    assert snap["present"].tolist() == [1, 1, 1, 1, 1]
