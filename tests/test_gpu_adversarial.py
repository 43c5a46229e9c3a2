"""cfg5 (sybil IP groups + invalid-message spam) on the GPU vs the CPU
oracle: scores after refresh and the state after two heartbeats, bit-exact."""
import numpy as np
import pytest

import adversarial_cases as ac
import gsx
import heartbeat_cases as hc
import oracle as orc
from gsx import abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2500, 12000])
def test_adversarial_matches_oracle(gpu_ok, n):
    res = []
    for be in (gsx.Engine(1), orc.Oracle(1)):
        ov = ac.setup(be, n, seed=n)
        snaps = [hc.snapshot(be)]
        for k in range(2):
            out = be.heartbeat(59 + k, ac.T0 + (2 + k) * abi.SECOND, 9).as_dict()
            be.refresh(ac.T0 + (2 + k) * abi.SECOND + 500 * abi.MILLISECOND)
            snaps.append((out, hc.snapshot(be)))
        res.append(snaps)
    g, w = res
    for f in list(abi.STATE_FIELDS) + ["scores"]:
        assert np.array_equal(np.asarray(g[0][f]).view(np.uint8), np.asarray(w[0][f]).view(np.uint8)), f
    for k in (1, 2):
        assert g[k][0] == w[k][0], k
        for f in list(abi.STATE_FIELDS) + ["backoff", "scores", "ihave_len", "ihave_digest"]:
            assert np.array_equal(np.asarray(g[k][1][f]).view(np.uint8), np.asarray(w[k][1][f]).view(np.uint8)), (k, f)
    assert g[1][0]["prunes"] > 0


def test_invalid_message_spam_stops_at_graylist(gpu_ok):
    """TestGossipsubAttackInvalidMessageSpam (gossipsub_spam_test.go:615-763)
    through the engine: 100 rejected single-message RPCs, the attacker is
    graylisted after the 4th (score -396 < -300) and every later RPC is dropped
    by AcceptFrom (tests/spam_cases.py); every call matches the oracle."""
    import spam_cases as sc

    e, o = gsx.Engine(1), orc.Oracle(1)
    g = sc.run(e)
    sc.check(g)
    assert g == sc.run(o)
    # the legit node PRUNEs the attacker once its score is negative
    # (gossipsub_spam_test.go:745-750): its heartbeat drops the negative-score
    # mesh peer (gossipsub.go:1361-1368) and sends PRUNE; the attacker is backed off
    hb = [sc.heartbeat(be) for be in (e, o)]
    sc.check_prune(hb[0])
    assert hb[0] == hb[1]
    assert e.export_backoff()[0][0] > sc.T0 + sc.S  # PRUNE backoff on the attacker
    assert np.array_equal(e.export_backoff(), o.export_backoff())
