"""Peer exchange on PRUNE on the GPU (k_hb_px through gsx_heartbeat) vs the CPU
oracle: round counters, the connection-candidate records, and the state the
round leaves (PX must not disturb it), bit-exact."""
import numpy as np
import pytest

import gsx
import oracle as orc
import px_cases as xc
from gsx import abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw", [dict(), dict(prune_peers=5), dict(leaf_view=-1.0), dict(no_px=True),
                                dict(n_leaves=16, hub_view={1: -5.0, 2: -5.0})])
def test_px_star_matches_oracle(gpu_ok, kw):
    g = xc.star_case(gsx.Engine(1), **kw)
    w = xc.star_case(orc.Oracle(1), **kw)
    assert g[0] == w[0]
    assert np.array_equal(g[1], w[1])


CASES = [
    # n, d, T, ticks, mesh_degree, d_hi, prune_peers, accept_px, join_frac, prop_msgs
    (400, 8, 2, 4, 3, 6, 4, 1.0, 0.85, 0),
    (600, 6, 1, 3, 14, 12, 16, 0.0, 1.0, 64),
    (800, 10, 2, 3, 4, 6, 16, 0.5, 0.9, 32),
]


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}-T{c[2]}-m{c[4]}-dhi{c[5]}" for c in CASES])
def test_px_rounds_match_oracle(gpu_ok, case):
    n, d, T, ticks, md, dhi, pp, acc, jf, pm = case
    runs = []
    for be in (gsx.Engine(T), orc.Oracle(T)):
        runs.append(xc.px_run(be, n, d, T, seed=n + d, ticks=ticks, mesh_degree=md, d_hi=dhi, prune_peers=pp,
                              accept_px=acc, join_frac=jf, prop_msgs=pm))
    (_, go, gr, gs), (_, wo, wr, ws) = runs
    for k in range(ticks):
        assert go[k] == wo[k], (k, go[k], wo[k])
        assert np.array_equal(gr[k], wr[k]), (k, len(gr[k]), len(wr[k]))
        for f in list(abi.STATE_FIELDS) + ["backoff", "scores", "ihave_len", "ihave_digest"]:
            x, y = np.asarray(gs[k][f]), np.asarray(ws[k][f])
            assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (k, f)
    assert sum(o["px_connect"] for o in go) > 0


def test_px_log_capacity_keeps_count(gpu_ok):
    out, rec, _ = xc.star_case(gsx.Engine(1), px_log=10)  # keeps 10 of the round's candidates, counts all
    full = xc.star_case(orc.Oracle(1))[1]
    assert out["px_connect"] == 104 and len(rec) == 10
    assert all(any((r == f).all() for f in full) for r in rec)


def test_px_member_rounds_match_oracle(gpu_ok):
    g = xc.px_member_run(gsx.Engine(2))
    w = xc.px_member_run(orc.Oracle(2))
    for (go, gr), (wo, wr) in zip(g, w):
        assert go == wo
        assert np.array_equal(gr, wr)
    assert g[1][0]["px_prunes"] > 0  # the Leave PRUNEs carried lists
