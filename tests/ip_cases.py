"""refreshIPs / setIPs cases (score.go:560-586, 1021-1059) on any backend: one
observer (node 0) with peers 1..5, IP colocation weight -1 above 1 peer per IP."""
import numpy as np

from gsx import abi

S = abi.SECOND
T0 = 1_700_000_000 * S
NO = abi.GSX_NO_IP


def setup(be):
    K = 5
    be.set_peer_params(abi.PeerScoreParams(ip_colocation_factor_weight=-1.0, ip_colocation_factor_threshold=1,
                                           app_specific_score_set=1, decay_interval_ns=S, decay_to_zero=0.01,
                                           retain_score_ns=10 * S))
    row_ptr = np.array([0] + [K] * (K + 1), dtype=np.int64)
    col = np.arange(1, K + 1, dtype=np.int32)
    ips = np.full((K + 1, 2), NO, dtype=np.uint32)
    ips[1:, 0] = [1, 2, 2, 2, 3]  # A on 1, B C D on 2, E on 3
    be.load_overlay(row_ptr, col, None, ips)
    return K


def ev(be, kind, p, now=T0):
    be.apply_events(np.array([(kind, 0, p, now, 0)], dtype=abi.event_dtype()))


def run(be):
    """-> list of score vectors after each step"""
    K = setup(be)
    out = []
    for p in range(4):  # A B C D connect; E stays absent
        ev(be, abi.EV_ADD_PEER, p)
    out.append(be.scores())                                   # B C D: (3-1)^2 = -4
    be.set_pair_ips([3], [[1, NO]])                          # D moves to A's IP: 1 -> {A, D}, 2 -> {B, C}
    out.append(be.scores())                                   # everyone -1
    be.set_pair_ips([4], [[2, 2]])                            # absent E: recorded, not counted
    out.append(be.scores())
    ev(be, abi.EV_ADD_PEER, 4)                                # AddPeer counts E on 2 (once: a set)
    out.append(be.scores())                                   # B C E on 2: -4 each, E's list has 2 twice: -8
    be.set_pair_ips([1, 2], [[7, NO], [NO, NO]])              # B to a new IP, C loses its address
    out.append(be.scores())
    be.apply_events(np.array([(abi.EV_REMOVE_PEER, 0, 0, T0, 0)], dtype=abi.event_dtype()))  # A retained (score < 0)
    be.set_pair_ips([0], [[3, NO]])                           # a retained peer moves too
    out.append(be.scores())
    return out, K
