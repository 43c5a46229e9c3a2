"""The gossip exchange on the GPU vs the CPU oracle (gsx.h heartbeat step (D):
handleIHave / handleIWant, gossipsub.go:615-716; promises and their P7
penalty, gossip_tracer.go:48-153, gossipsub.go:1578-1583): every round's
counters, records, scores (P7 through behaviourPenalty), IHAVEs and every
node's cached ids (the recovered copies) are equal."""
import numpy as np
import pytest

import gossip_cases as gc
import gsx
import oracle as orc
from gsx import abi

pytestmark = pytest.mark.gpu

FIELDS = list(abi.STATE_FIELDS) + ["backoff", "scores", "ihave_len", "ihave_digest"]


def _same(g, w):
    ov, go, gs, gcache = g
    _, wo, ws, wcache = w
    for k in range(len(go)):  # the first tick that differs: its counters, then its state
        diff = {x: (go[k][x], wo[k][x]) for x in go[k] if go[k][x] != wo[k][x]}
        assert not diff, f"tick {k}: {diff}"
        for f in FIELDS:
            a, b = np.asarray(gs[k][f]), np.asarray(ws[k][f])
            if not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                bad = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
                pytest.fail(f"tick {k} field {f}: {len(bad)} differ, first {bad[:5].tolist()} "
                            f"gpu {a.reshape(-1)[bad[:5]].tolist()} oracle {b.reshape(-1)[bad[:5]].tolist()}")
    for v, (a, b) in enumerate(zip(gcache, wcache)):
        assert sorted(a.tolist()) == sorted(b.tolist()), v


@pytest.mark.parametrize("kw", [
    dict(),                                   # HistoryGossip == HistoryLength (reference default)
    dict(history_gossip=3),                   # everything asked is served
    dict(exchange_from=5, ticks=10),          # unanswered IHAVEs: broken promises, P7
    dict(invalid=0.3, ticks=6),               # recovered invalid messages: P4
    dict(T=1, n=500, d=8, msgs=70, ticks=6),  # two words per batch
])
def test_gossip_exchange_matches_oracle(gpu_ok, kw):
    T = kw.get("T", 2)
    g = gc.exchange_run(gsx.Engine(T), **kw)
    w = gc.exchange_run(orc.Oracle(T), **kw)
    _same(g, w)
    assert sum(o["iwant_msgs"] for o in g[1]) > 0
