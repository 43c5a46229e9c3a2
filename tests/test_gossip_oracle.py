"""The gossip exchange of the CPU oracle (gsx.h heartbeat step (D)):
handleIHave / handleIWant (gossipsub.go:615-716), promise tracking and the
P7 penalty for broken promises (gossip_tracer.go:48-153, gossipsub.go:1578-1583)."""
import numpy as np
import pytest

import gossip_cases as gc
import oracle as orc
from gsx import abi


def test_exchange_recovers_missed_messages():
    ov, outs, snaps, cached = gc.exchange_run(orc.Oracle(2))
    tot = {k: sum(o[k] for o in outs) for k in outs[0]}
    assert tot["iwant_msgs"] > 0 and tot["iwant_ids"] >= tot["iwant_msgs"]
    assert 0 < tot["iwant_served"] <= tot["iwant_ids"]
    assert tot["gossip_delivered"] > 0
    # a served message is received once (delivered / rejected) or as a duplicate
    assert tot["gossip_delivered"] + tot["gossip_rejected"] + tot["gossip_duplicates"] == tot["iwant_served"]


def test_exchange_off_changes_nothing():
    _, outs, _, _ = gc.exchange_run(orc.Oracle(2), gossip_exchange=0)
    for o in outs:
        assert o["iwant_msgs"] == o["gossip_delivered"] == o["broken_promises"] == 0


def test_oldest_window_is_not_served_and_promises_break():
    """HistoryGossip == HistoryLength (the reference default, gossipsub.go:238):
    the IHAVE advertises the window the Shift drops before the IWANT arrives,
    so some asks go unanswered; promises on them expire after
    IWantFollowupTime and AddPenalty raises P7 of the advertiser."""
    be = orc.Oracle(2)
    ov, outs, snaps, _ = gc.exchange_run(be, ticks=10, exchange_from=5)  # five windows of unanswered IHAVEs
    assert outs[5]["iwant_served"] < outs[5]["iwant_ids"]
    # expiry now + 3 s: broken at the first heartbeat strictly after it (4 ticks later)
    assert sum(o["broken_promises"] for o in outs[6:9]) == 0 and outs[9]["broken_promises"] > 0
    assert snaps[-1]["behaviour_penalty"].sum() > snaps[5]["behaviour_penalty"].sum()


def test_history_gossip_3_serves_everything():
    """HistoryGossip 3 < HistoryLength 5: every asked message is still cached
    when the IWANT arrives, every promise is kept."""
    _, outs, _, _ = gc.exchange_run(orc.Oracle(2), history_gossip=3, ticks=10)
    tot = {k: sum(o[k] for o in outs) for k in outs[0]}
    assert tot["iwant_ids"] > 0 and tot["iwant_served"] == tot["iwant_ids"]
    assert tot["broken_promises"] == 0


def test_low_scores_get_no_gossip_handled():
    """IHAVEs from peers below GossipThreshold are ignored (:617-621): with the
    threshold above every score nothing is asked."""
    be = orc.Oracle(2)
    _, outs, _, _ = gc.exchange_run(be, ticks=4, max_ihave_messages=0)  # peerhave limit: every RPC ignored
    assert sum(o["iwant_msgs"] for o in outs) == 0 and sum(o["ihave_ignored"] for o in outs) > 0


def test_invalid_messages_recovered_are_rejected():
    _, outs, _, _ = gc.exchange_run(orc.Oracle(2), invalid=0.3, ticks=8)
    tot = {k: sum(o[k] for o in outs) for k in outs[0]}
    assert tot["gossip_delivered"] > 0


def test_recovered_copies_are_cached():
    """A recovered message is Put into the node's cache (window 0 after the Shift)."""
    be = orc.Oracle(2)
    ov, outs, snaps, cached = gc.exchange_run(be, ticks=3, history_gossip=3)
    assert outs[-1]["gossip_delivered"] > 0
    n_cached = sum(len(c) for c in cached)
    be2 = orc.Oracle(2)
    _, _, _, cached2 = gc.exchange_run(be2, ticks=3, history_gossip=3, gossip_exchange=0)
    assert n_cached > sum(len(c) for c in cached2)


def test_exchange_window_boundary_between_hops_splits_credits():
    """The oracle keeps each node's validation time (score.go:944-974): with the
    P3 window boundary between arrival hops (892 ms: hop 2 of the last batch
    inside, hops 0-1 outside) the forwarded duplicates' MMD credits differ from
    both a window that leaves every old copy outside (880 ms) and one that
    takes every copy of the last batch in (905 ms)."""
    mmd = {}
    for win in (880, 892, 905):
        _, outs, snaps, _ = gc.exchange_run(orc.Oracle(2), window_ms=win, hops=3, ticks=5)
        assert sum(o["fwd_duplicates"] for o in outs) > 0
        mmd[win] = np.concatenate([np.asarray(s["mesh_message_deliveries"]).reshape(-1) for s in snaps])
    assert not np.array_equal(mmd[892], mmd[880])
    assert not np.array_equal(mmd[892], mmd[905])
