"""Topic membership on the GPU vs the CPU oracle (gsx.h): partial
subscriptions as the "in topic" filter, fanout publishing for publishers that
have not joined (gossipsub.go:981-998), the heartbeat's fanout expiry and
maintenance (:1517-1554), Join / Leave (:1015-1082).  Every round's counters,
records, scores, backoff, IHAVEs, membership (joined, fanout, lastpub) and
propagation outcomes are equal."""
import numpy as np
import pytest

import gsx
import membership_cases as mc
import oracle as orc
from gsx import abi

pytestmark = pytest.mark.gpu

FIELDS = list(abi.STATE_FIELDS) + ["backoff", "scores", "ihave_len", "ihave_digest"]


@pytest.mark.parametrize("kw", [dict(), dict(T=1, n=600, d=8, fanout_ttl_s=1), dict(T=4, ticks=7, msgs=40)])
def test_membership_matches_oracle(gpu_ok, kw):
    T = kw.get("T", 2)
    g = mc.membership_run(gsx.Engine(T), **kw)
    w = mc.membership_run(orc.Oracle(T), **kw)
    _, go, gs, gm, gp = g
    _, wo, ws, wm, wp = w
    assert len(go) == len(wo)
    for k, (a, b) in enumerate(zip(go, wo)):
        diff = {x: (a[1][x], b[1][x]) for x in a[1] if a[1][x] != b[1][x]}
        assert a[0] == b[0] and not diff, f"step {k} ({a[0]}): {diff}"
    for k in range(len(gs)):
        for f in FIELDS:
            x, y = np.asarray(gs[k][f]), np.asarray(ws[k][f])
            assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (k, f)
        for name, x, y in zip(("joined", "fanout", "lastpub"), gm[k], wm[k]):
            assert np.array_equal(x, y), (k, name)
        assert gp[k][0] == wp[k][0], k
        assert np.array_equal(gp[k][1], wp[k][1]), k
    assert any(np.count_nonzero(m[1]) for m in gm)  # some fanout was used
