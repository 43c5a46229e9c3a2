"""TestGossipsubAttackInvalidMessageSpam (gossipsub_spam_test.go:615-763)
restated for the synchronous engine: a legit gossipsub node (0) and an
attacker (1) meshed on one topic; the attacker publishes 100 messages that
fail validation, one RPC (one propagation call) each, with the test's own
parameters (:627-660).  Every rejected message adds one invalid delivery
(P4); after the 4th the attacker's score is 16 * -99 * 0.25 = -396 <
GraylistThreshold -300, so gossipsub's AcceptFrom (gossipsub.go:583-594)
makes the legit node drop every later RPC before pushMsg
(pubsub.go:1014-1017): the invalid count stops at 4 instead of reaching 100.
Loaded identically into any backend (engine or oracle)."""
from __future__ import annotations

import numpy as np

from gsx import abi

S = abi.SECOND
T0 = 1_700_000_000 * S
N_MSGS = 100


def peer_params() -> abi.PeerScoreParams:
    """gossipsub_spam_test.go:627-635 (AppSpecificScore returns 0)."""
    return abi.PeerScoreParams(topic_score_cap=0.0, app_specific_weight=0.0, app_specific_score_set=1,
                               ip_colocation_factor_threshold=1, ip_colocation_factor_weight=0.0,
                               behaviour_penalty_weight=0.0, behaviour_penalty_threshold=0.0,
                               behaviour_penalty_decay=0.0, decay_interval_ns=5 * S, decay_to_zero=0.01,
                               retain_score_ns=10 * S)


THRESHOLDS = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                            accept_px_threshold=0, opportunistic_graft_threshold=0)


def setup(be):
    from gsx import synth

    be.set_peer_params(peer_params())
    be.set_topic_params(0, synth.spam_test_topic_params())
    be.set_thresholds(THRESHOLDS)
    row_ptr = np.array([0, 1, 2], dtype=np.int64)
    col = np.array([1, 0], dtype=np.int32)
    ef = np.array([abi.GSX_EDGE_GOSSIPSUB | abi.GSX_EDGE_OUTBOUND, abi.GSX_EDGE_GOSSIPSUB], dtype=np.uint8)
    ips = np.array([[1, 0xFFFFFFFF], [2, 0xFFFFFFFF]], dtype=np.uint32)
    be.load_overlay(row_ptr, col, ef, ips)
    be.set_app_scores(np.zeros(2))
    # connect, then the attacker's GRAFT is accepted (handleGraft, score 0) and
    # the attacker keeps the legit node in its own mesh
    ev = [(abi.EV_ADD_PEER, 0, 0, T0, 0), (abi.EV_ADD_PEER, 0, 1, T0, 0),
          (abi.EV_GRAFT, 0, 0, T0, 0), (abi.EV_GRAFT, 0, 1, T0, 0)]
    be.apply_events(np.array(ev, dtype=abi.event_dtype()))


def run(be):
    """-> per-call rows (rejected, graylisted, invalid count of the legit node's
    record of the attacker, its score after the call)."""
    setup(be)
    rows = []
    for i in range(N_MSGS):
        ms = np.zeros(1, dtype=abi.msg_dtype())
        ms["source"] = 1
        ms["validation"] = abi.GSX_VALIDATION_REJECT
        ms["msg_id"] = i + 1
        cfg = abi.PropConfig(router=abi.GSX_ROUTER_GOSSIPSUB, topic=0, flood_publish=0, max_hops=4,
                             hop_latency_ns=abi.MILLISECOND, now_ns=T0 + i * abi.MILLISECOND,
                             credit_scores=abi.GSX_CREDIT_NOW, randomsub_size=0, seed=1, validation_delay_ns=0)
        out, _, _ = be.propagate(ms, cfg)
        st = be.export_state()
        rows.append((int(out.rejected), int(out.graylisted), float(st["invalid_message_deliveries"][0]),
                     float(be.scores()[0])))
    return rows


def heartbeat(be):
    """The legit node's first heartbeat after the spam (gossipsub_spam_test.go:
    728-750: wait for GossipSubHeartbeatInitialDelay + 100 ms, then the
    attacker's score is below zero and the legit node has sent a PRUNE):
    (A) prunes a negative-score mesh peer (gossipsub.go:1361-1368).  Returns
    (the round's counters, the attacker's score at the legit node before the
    round, whether it is still in the legit node's mesh, the topics of the
    PRUNEs the legit node sent to it)."""
    before = float(be.scores()[0])
    be.hb_set_tracing(True)
    now = T0 + N_MSGS * abi.MILLISECOND + 200 * abi.MILLISECOND  # initial delay (gossipsub.go:44) + 100 ms
    out = be.heartbeat(1, now, 1).as_dict()
    st = be.export_state()
    in_mesh = bool(st["rec_flags"][0] & abi.GSX_REC_IN_MESH)  # pair 0: the legit node's record of the attacker
    sent_prune = int(be.hb_trace_words()[1][0])
    return out, before, in_mesh, sent_prune


def check_prune(res):
    """The reference test's last assertion: the legit node PRUNEs the attacker
    once its score is negative (gossipsub_spam_test.go:743-750)."""
    out, before, in_mesh, sent_prune = res
    assert before < 0
    assert out["prunes"] == 1 and sent_prune == 1  # one PRUNE, topic 0, on the legit node's pair
    assert not in_mesh


def check(rows):
    """The reference test's assertions plus the graylist cut-off."""
    assert [r[0] for r in rows[:4]] == [1, 1, 1, 1]
    assert all(r[0] == 0 and r[1] == 1 for r in rows[4:])  # dropped by AcceptFrom
    assert [r[2] for r in rows[:4]] == [1.0, 2.0, 3.0, 4.0]
    assert all(r[2] == 4.0 for r in rows[4:])  # the invalid count stops at 4, not 100
    assert [r[3] for r in rows[:4]] == [-24.75, -99.0, -222.75, -396.0]
    assert rows[-1][3] == -396.0 < THRESHOLDS.graylist_threshold
    assert sum(r[0] for r in rows) == 4  # tracer.rejectCount (REJECT_MESSAGE events)
