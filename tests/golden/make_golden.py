"""Generates the known-answer fixtures of tests/golden/ from the reference's own tests.

The reference is Go and cannot be built or run in this container (no Go
toolchain), so its known answers are taken from the expected
values its unit tests assert.  Each scenario below restates one test of
/root/reference/score_test.go (or score_params_test.go) as data: the calls the
test makes, in order, and the values it asserts.  Expected numbers are computed
here with the test's own expression, in its own operation order, in IEEE
binary64 (Python floats == Go float64 on amd64).

Wall-clock sleeps of the Go tests become explicit advances of a simulated
clock (the engine takes `now` as an argument).  Where the Go test can only
assert an inequality because of real sleeps (TimeInMesh ">=", TimeInMeshCap
"within 50 %", MeshMessageDeliveries "non-negative"), the fixture records the
exact value the same expression gives under the simulated clock and keeps the
Go relation in `go_assert` for reference.

Run:  python tests/golden/make_golden.py
      (writes score_kat.json, params_validation.json, promise_kat.json)
"""
from __future__ import annotations

import json
import math
import os

S = 1_000_000_000
MS = 1_000_000
HOUR = 3600 * S
INF = float("inf")
NAN = float("nan")

OUT = os.path.dirname(os.path.abspath(__file__))


def topic(**kw):
    """TopicScoreParams with Go zero values for unset fields."""
    base = dict(
        topic_weight=0.0,
        time_in_mesh_weight=0.0,
        time_in_mesh_quantum_ns=0,
        time_in_mesh_cap=0.0,
        first_message_deliveries_weight=0.0,
        first_message_deliveries_decay=0.0,
        first_message_deliveries_cap=0.0,
        mesh_message_deliveries_weight=0.0,
        mesh_message_deliveries_decay=0.0,
        mesh_message_deliveries_cap=0.0,
        mesh_message_deliveries_threshold=0.0,
        mesh_message_deliveries_window_ns=0,
        mesh_message_deliveries_activation_ns=0,
        mesh_failure_penalty_weight=0.0,
        mesh_failure_penalty_decay=0.0,
        invalid_message_deliveries_weight=0.0,
        invalid_message_deliveries_decay=0.0,
    )
    for k, v in kw.items():
        assert k in base, k
        base[k] = v
    return base


def peer(**kw):
    """PeerScoreParams (non-map fields) with Go zero values; AppSpecificScore set."""
    base = dict(
        topic_score_cap=0.0,
        app_specific_weight=0.0,
        app_specific_score_set=1,
        ip_colocation_factor_threshold=0,
        ip_colocation_factor_weight=0.0,
        behaviour_penalty_weight=0.0,
        behaviour_penalty_threshold=0.0,
        behaviour_penalty_decay=0.0,
        decay_interval_ns=0,
        decay_to_zero=0.0,
        retain_score_ns=0,
    )
    for k, v in kw.items():
        assert k in base, k
        base[k] = v
    return base


def thr(**kw):
    base = dict(
        gossip_threshold=0.0,
        publish_threshold=0.0,
        graylist_threshold=0.0,
        accept_px_threshold=0.0,
        opportunistic_graft_threshold=0.0,
    )
    base.update(kw)
    return base


def scenarios():
    out = []
    T = "mytopic"

    # TestScoreTimeInMesh, score_test.go:13-50
    tp = topic(topic_weight=0.5, time_in_mesh_weight=1, time_in_mesh_quantum_ns=MS, time_in_mesh_cap=3600)
    elapsed = 200 * MS
    exp = tp["topic_weight"] * tp["time_in_mesh_weight"] * float(elapsed // tp["time_in_mesh_quantum_ns"])
    out.append(dict(
        name="TestScoreTimeInMesh", ref="score_test.go:13-50", topic_params={T: tp}, peer_params=peer(),
        peers=["A"], go_assert="score >= expected (real sleep); exact under the simulated clock",
        steps=[["add_peer", "A"], ["expect_score", "A", 0.0], ["graft", "A", T], ["advance", elapsed],
               ["refresh"], ["expect_score", "A", exp]]))

    # TestScoreTimeInMeshCap, score_test.go:52-84
    tp = topic(topic_weight=0.5, time_in_mesh_weight=1, time_in_mesh_quantum_ns=MS, time_in_mesh_cap=10)
    exp = tp["topic_weight"] * tp["time_in_mesh_weight"] * tp["time_in_mesh_cap"]
    out.append(dict(
        name="TestScoreTimeInMeshCap", ref="score_test.go:52-84", topic_params={T: tp}, peer_params=peer(),
        peers=["A"], go_assert="within 50% of expected (real sleep); exact under the simulated clock",
        steps=[["add_peer", "A"], ["graft", "A", T], ["advance", 40 * MS], ["refresh"], ["expect_score", "A", exp]]))

    # TestScoreFirstMessageDeliveries / Cap / Decay, score_test.go:86-215
    for name, ref, cap, dec in [
        ("TestScoreFirstMessageDeliveries", "score_test.go:86-124", 2000, 1.0),
        ("TestScoreFirstMessageDeliveriesCap", "score_test.go:126-164", 50, 1.0),
        ("TestScoreFirstMessageDeliveriesDecay", "score_test.go:166-215", 2000, 0.9),
    ]:
        tp = topic(topic_weight=1, first_message_deliveries_weight=1, first_message_deliveries_decay=dec,
                   first_message_deliveries_cap=cap, time_in_mesh_quantum_ns=S)
        steps = [["add_peer", "A"], ["graft", "A", T]]
        for i in range(100):
            steps += [["validate", "A", i, T], ["deliver", "A", i, T]]
        steps += [["refresh"]]
        if name.endswith("Decay"):
            exp = tp["topic_weight"] * tp["first_message_deliveries_weight"] * tp["first_message_deliveries_decay"] * float(100)
            steps += [["expect_score", "A", exp]]
            for _ in range(10):
                steps += [["refresh"]]
                exp *= tp["first_message_deliveries_decay"]
            steps += [["expect_score", "A", exp]]
        elif name.endswith("Cap"):
            steps += [["expect_score", "A", tp["topic_weight"] * tp["first_message_deliveries_weight"] * tp["first_message_deliveries_cap"]]]
        else:
            steps += [["expect_score", "A", tp["topic_weight"] * tp["first_message_deliveries_weight"] * float(100)]]
        out.append(dict(name=name, ref=ref, topic_params={T: tp}, peer_params=peer(), peers=["A"], steps=steps))

    # TestScoreMeshMessageDeliveries, score_test.go:217-308
    tp = topic(topic_weight=1, mesh_message_deliveries_weight=-1, mesh_message_deliveries_activation_ns=S,
               mesh_message_deliveries_window_ns=10 * MS, mesh_message_deliveries_threshold=20,
               mesh_message_deliveries_cap=100, mesh_message_deliveries_decay=1.0,
               first_message_deliveries_weight=0, time_in_mesh_quantum_ns=S)
    steps = []
    for p in "ABC":
        steps += [["add_peer", p], ["graft", p, T]]
    steps += [["refresh"], ["expect_score_ge", "A", 0.0], ["expect_score_ge", "B", 0.0], ["expect_score_ge", "C", 0.0],
              ["advance", S]]
    for i in range(100):
        steps += [["validate", "A", i, T], ["deliver", "A", i, T], ["duplicate", "B", i, T]]
    steps += [["advance", 10 * MS + 20 * MS]]
    for i in range(100):
        steps += [["duplicate", "C", i, T]]
    penalty = tp["mesh_message_deliveries_threshold"] * tp["mesh_message_deliveries_threshold"]
    exp = tp["topic_weight"] * tp["mesh_message_deliveries_weight"] * penalty
    steps += [["refresh"], ["expect_score", "A", 0.0], ["expect_score", "B", 0.0], ["expect_score", "C", exp]]
    out.append(dict(name="TestScoreMeshMessageDeliveries", ref="score_test.go:217-308", topic_params={T: tp},
                    peer_params=peer(), peers=["A", "B", "C"],
                    go_assert="A, B >= 0 (exactly 0 here); C == expected", steps=steps))

    # TestScoreMeshMessageDeliveriesDecay, score_test.go:310-369
    tp = topic(topic_weight=1, mesh_message_deliveries_weight=-1, mesh_message_deliveries_activation_ns=0,
               mesh_message_deliveries_window_ns=10 * MS, mesh_message_deliveries_threshold=20,
               mesh_message_deliveries_cap=100, mesh_message_deliveries_decay=0.9,
               first_message_deliveries_weight=0, time_in_mesh_quantum_ns=S)
    steps = [["add_peer", "A"], ["graft", "A", T]]
    for i in range(40):
        steps += [["validate", "A", i, T], ["deliver", "A", i, T]]
    steps += [["advance", MS], ["refresh"], ["expect_score_ge", "A", 0.0]]
    dc = float(40) * tp["mesh_message_deliveries_decay"]
    for _ in range(20):
        steps += [["refresh"]]
        dc *= tp["mesh_message_deliveries_decay"]
    deficit = tp["mesh_message_deliveries_threshold"] - dc
    exp = tp["topic_weight"] * tp["mesh_message_deliveries_weight"] * (deficit * deficit)
    steps += [["expect_score", "A", exp]]
    out.append(dict(name="TestScoreMeshMessageDeliveriesDecay", ref="score_test.go:310-369", topic_params={T: tp},
                    peer_params=peer(), peers=["A"], steps=steps))

    # TestScoreMeshFailurePenalty, score_test.go:371-450
    tp = topic(topic_weight=1, mesh_failure_penalty_weight=-1, mesh_failure_penalty_decay=1.0,
               mesh_message_deliveries_activation_ns=0, mesh_message_deliveries_window_ns=10 * MS,
               mesh_message_deliveries_threshold=20, mesh_message_deliveries_cap=100,
               mesh_message_deliveries_decay=1.0, mesh_message_deliveries_weight=0,
               first_message_deliveries_weight=0, time_in_mesh_quantum_ns=S)
    steps = []
    for p in "AB":
        steps += [["add_peer", p], ["graft", p, T]]
    for i in range(100):
        steps += [["validate", "A", i, T], ["deliver", "A", i, T]]
    steps += [["advance", MS], ["refresh"], ["expect_score", "A", 0.0], ["expect_score", "B", 0.0],
              ["prune", "B", T], ["refresh"], ["expect_score", "A", 0.0]]
    penalty = tp["mesh_message_deliveries_threshold"] * tp["mesh_message_deliveries_threshold"]
    steps += [["expect_score", "B", tp["topic_weight"] * tp["mesh_failure_penalty_weight"] * penalty]]
    out.append(dict(name="TestScoreMeshFailurePenalty", ref="score_test.go:371-450", topic_params={T: tp},
                    peer_params=peer(), peers=["A", "B"], steps=steps))

    # TestScoreInvalidMessageDeliveries, score_test.go:452-487
    tp = topic(topic_weight=1, time_in_mesh_quantum_ns=S, invalid_message_deliveries_weight=-1,
               invalid_message_deliveries_decay=1.0)
    steps = [["add_peer", "A"], ["graft", "A", T]]
    for i in range(100):
        steps += [["reject", "A", i, T, "invalid signature"]]
    steps += [["refresh"], ["expect_score", "A", tp["topic_weight"] * tp["invalid_message_deliveries_weight"] * float(100 * 100)]]
    out.append(dict(name="TestScoreInvalidMessageDeliveries", ref="score_test.go:452-487", topic_params={T: tp},
                    peer_params=peer(), peers=["A"], steps=steps))

    # TestScoreInvalidMessageDeliveriesDecay, score_test.go:489-534
    tp = topic(topic_weight=1, time_in_mesh_quantum_ns=S, invalid_message_deliveries_weight=-1,
               invalid_message_deliveries_decay=0.9)
    steps = [["add_peer", "A"], ["graft", "A", T]]
    for i in range(100):
        steps += [["reject", "A", i, T, "invalid signature"]]
    exp = tp["topic_weight"] * tp["invalid_message_deliveries_weight"] * math.pow(tp["invalid_message_deliveries_decay"] * float(100), 2)
    steps += [["refresh"], ["expect_score", "A", exp]]
    for _ in range(10):
        steps += [["refresh"]]
        exp *= math.pow(tp["invalid_message_deliveries_decay"], 2)
    steps += [["expect_score", "A", exp]]
    out.append(dict(name="TestScoreInvalidMessageDeliveriesDecay", ref="score_test.go:489-534", topic_params={T: tp},
                    peer_params=peer(), peers=["A"], steps=steps))

    # TestScoreRejectMessageDeliveries, score_test.go:536-666
    tp = topic(topic_weight=1, time_in_mesh_quantum_ns=S, invalid_message_deliveries_weight=-1,
               invalid_message_deliveries_decay=1.0)
    m = 0
    steps = [["add_peer", "A"], ["add_peer", "B"],
             ["reject", "A", m, T, "blacklisted peer"], ["reject", "A", m, T, "blacklisted source"],
             ["reject", "A", m, T, "validation queue full"], ["expect_score", "A", 0.0],
             ["validate", "A", m, T], ["reject", "A", m, T, "validation throttled"], ["duplicate", "B", m, T],
             ["expect_score", "A", 0.0], ["expect_score", "B", 0.0],
             ["gc_expire_all"],
             ["validate", "A", m, T], ["reject", "A", m, T, "validation ignored"], ["duplicate", "B", m, T],
             ["expect_score", "A", 0.0], ["expect_score", "B", 0.0],
             ["gc_expire_all"],
             ["validate", "A", m, T], ["reject", "A", m, T, "validation failed"], ["duplicate", "B", m, T],
             ["expect_score", "A", -1.0], ["expect_score", "B", -1.0],
             ["gc_expire_all"],
             ["validate", "A", m, T], ["duplicate", "B", m, T], ["reject", "A", m, T, "validation failed"],
             ["expect_score", "A", -4.0], ["expect_score", "B", -4.0]]
    out.append(dict(name="TestScoreRejectMessageDeliveries", ref="score_test.go:536-666", topic_params={T: tp},
                    peer_params=peer(), peers=["A", "B"],
                    go_assert="the test forces gc by setting head.expire=now; here the clock jumps past TimeCacheDuration",
                    steps=steps))

    # TestScoreApplicationScore, score_test.go:668-694 (no topic params: graft is a no-op)
    steps = [["add_peer", "A"], ["graft", "A", T]]
    for i in range(-100, 100):
        steps += [["set_app", "A", float(i)], ["refresh"], ["expect_score", "A", float(i) * 0.5]]
    out.append(dict(name="TestScoreApplicationScore", ref="score_test.go:668-694", topic_params={},
                    peer_params=peer(app_specific_weight=0.5), peers=["A"], steps=steps))

    # TestScoreIPColocation / Whitelist, score_test.go:696-803
    ips = {"A": ["1.2.3.4"], "B": ["2.3.4.5"], "C": ["2.3.4.5", "3.4.5.6"], "D": ["2.3.4.5"]}
    pp = peer(ip_colocation_factor_threshold=1, ip_colocation_factor_weight=-1)
    steps = []
    for p in "ABCD":
        steps += [["add_peer", p], ["graft", p, T]]
    n_shared = 3
    surplus = n_shared - pp["ip_colocation_factor_threshold"]
    exp = pp["ip_colocation_factor_weight"] * float(surplus * surplus)
    out.append(dict(name="TestScoreIPColocation", ref="score_test.go:696-744", topic_params={}, peer_params=pp,
                    peers=list("ABCD"), ips=ips,
                    go_assert="IPs injected with setIPsForPeer after AddPeer; here they are known at AddPeer (same final peerIPs)",
                    steps=steps + [["refresh"], ["expect_score", "A", 0.0], ["expect_score", "B", exp],
                                   ["expect_score", "C", exp], ["expect_score", "D", exp]]))
    out.append(dict(name="TestScoreIPColocationWhitelist", ref="score_test.go:746-803", topic_params={},
                    peer_params=pp, peers=list("ABCD"), ips=ips, whitelist_cidr="2.3.0.0/16",
                    steps=steps + [["refresh"]] + [["expect_score", p, 0.0] for p in "ABCD"]))

    # TestScoreBehaviourPenalty, score_test.go:805-859 (the nil-receiver part is N/A: no engine)
    pp = peer(behaviour_penalty_weight=-1, behaviour_penalty_decay=0.99)
    out.append(dict(name="TestScoreBehaviourPenalty", ref="score_test.go:805-859", topic_params={}, peer_params=pp,
                    peers=["A"],
                    steps=[["penalty", "A", 1], ["expect_score", "A", 0.0], ["add_peer", "A"], ["expect_score", "A", 0.0],
                           ["penalty", "A", 1], ["expect_score", "A", -1.0], ["penalty", "A", 1],
                           ["expect_score", "A", -4.0], ["refresh"], ["expect_score", "A", -3.9204]]))

    # TestScoreRetention, score_test.go:861-903
    pp = peer(app_specific_weight=1.0, retain_score_ns=S)
    out.append(dict(name="TestScoreRetention", ref="score_test.go:861-903", topic_params={}, peer_params=pp,
                    peers=["A"], app={"A": -1000.0},
                    steps=[["add_peer", "A"], ["graft", "A", T], ["refresh"], ["expect_score", "A", -1000.0],
                           ["remove_peer", "A"], ["advance", S // 2], ["refresh"], ["expect_score", "A", -1000.0],
                           ["advance", S // 2 + 50 * MS], ["refresh"], ["expect_score", "A", 0.0]]))

    # TestScoreRecapTopicParams, score_test.go:905-1000
    tp = topic(topic_weight=1, mesh_message_deliveries_weight=-1, mesh_message_deliveries_activation_ns=S,
               mesh_message_deliveries_window_ns=10 * MS, mesh_message_deliveries_threshold=20,
               mesh_message_deliveries_cap=100, mesh_message_deliveries_decay=1.0,
               first_message_deliveries_weight=10, first_message_deliveries_decay=1.0,
               first_message_deliveries_cap=100, time_in_mesh_quantum_ns=S)
    tp2 = dict(tp, mesh_message_deliveries_cap=50, first_message_deliveries_cap=50)
    steps = []
    for p in "AB":
        steps += [["add_peer", p], ["graft", p, T]]
    for i in range(100):
        steps += [["validate", "A", i, T], ["deliver", "A", i, T], ["duplicate", "B", i, T]]
    steps += [["expect_counter", "A", T, "first_message_deliveries", 100.0],
              ["expect_counter", "B", T, "mesh_message_deliveries", 100.0],
              ["set_topic_params", T, tp2],
              ["expect_counter", "A", T, "first_message_deliveries", 50.0],
              ["expect_counter", "B", T, "mesh_message_deliveries", 50.0]]
    out.append(dict(name="TestScoreRecapTopicParams", ref="score_test.go:905-1000", topic_params={T: tp},
                    peer_params=peer(), peers=["A", "B"], steps=steps))

    # TestScoreResetTopicParams, score_test.go:1002-1062
    tp = topic(topic_weight=1, time_in_mesh_quantum_ns=S, invalid_message_deliveries_weight=-1,
               invalid_message_deliveries_decay=1.0)
    tp2 = dict(tp, invalid_message_deliveries_weight=-10)
    steps = [["add_peer", "A"]]
    for i in range(100):
        steps += [["validate", "A", i, T], ["reject", "A", i, T, "validation failed"]]
    steps += [["expect_score", "A", -10000.0], ["set_topic_params", T, tp2], ["expect_score", "A", -100000.0]]
    out.append(dict(name="TestScoreResetTopicParams", ref="score_test.go:1002-1062", topic_params={T: tp},
                    peer_params=peer(), peers=["A"], steps=steps))
    return out


def _enc(x):
    """JSON cannot hold inf/nan: encode them as strings."""
    if isinstance(x, float) and (math.isinf(x) or math.isnan(x)):
        return repr(x)
    if isinstance(x, dict):
        return {k: _enc(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_enc(v) for v in x]
    return x


def validation_cases():
    """score_params_test.go: every case, with the verdict the test asserts."""
    cases = []
    # TestPeerScoreThresholdsValidation, score_params_test.go:11-49
    th = [
        (thr(gossip_threshold=1), False),
        (thr(publish_threshold=1), False),
        (thr(gossip_threshold=-1, publish_threshold=0), False),
        (thr(gossip_threshold=-1, publish_threshold=-2, graylist_threshold=0), False),
        (thr(accept_px_threshold=-1), False),
        (thr(opportunistic_graft_threshold=-1), False),
        (thr(gossip_threshold=-1, publish_threshold=-2, graylist_threshold=-3, accept_px_threshold=1, opportunistic_graft_threshold=2), True),
        (thr(gossip_threshold=-INF, publish_threshold=-2, graylist_threshold=-3, accept_px_threshold=1, opportunistic_graft_threshold=2), False),
        (thr(gossip_threshold=-1, publish_threshold=-INF, graylist_threshold=-3, accept_px_threshold=1, opportunistic_graft_threshold=2), False),
        (thr(gossip_threshold=-1, publish_threshold=-2, graylist_threshold=-INF, accept_px_threshold=1, opportunistic_graft_threshold=2), False),
        (thr(gossip_threshold=-1, publish_threshold=-2, graylist_threshold=-3, accept_px_threshold=NAN, opportunistic_graft_threshold=2), False),
        (thr(gossip_threshold=-1, publish_threshold=-2, graylist_threshold=-3, accept_px_threshold=1, opportunistic_graft_threshold=INF), False),
    ]
    for i, (p, ok) in enumerate(th):
        cases.append(dict(kind="thresholds", ref=f"score_params_test.go:11-49 #{i}", params=p, valid=ok))
    # TestTopicScoreParamsValidation, score_params_test.go:51-146
    good = topic(topic_weight=1, time_in_mesh_weight=0.01, time_in_mesh_quantum_ns=S, time_in_mesh_cap=10,
                 first_message_deliveries_weight=1, first_message_deliveries_decay=0.5, first_message_deliveries_cap=10,
                 mesh_message_deliveries_weight=-1, mesh_message_deliveries_decay=0.5, mesh_message_deliveries_cap=10,
                 mesh_message_deliveries_threshold=5, mesh_message_deliveries_window_ns=MS,
                 mesh_message_deliveries_activation_ns=S, mesh_failure_penalty_weight=-1, mesh_failure_penalty_decay=0.5,
                 invalid_message_deliveries_weight=-1, invalid_message_deliveries_decay=0.5)
    q = dict(time_in_mesh_quantum_ns=S)
    tps = [
        (topic(), False),
        (topic(topic_weight=-1), False),
        (topic(time_in_mesh_weight=-1, time_in_mesh_quantum_ns=S), False),
        (topic(time_in_mesh_weight=1, time_in_mesh_quantum_ns=-1), False),
        (topic(time_in_mesh_weight=1, time_in_mesh_quantum_ns=S, time_in_mesh_cap=-1), False),
        (topic(first_message_deliveries_weight=-1, **q), False),
        (topic(first_message_deliveries_weight=1, first_message_deliveries_decay=-1, **q), False),
        (topic(first_message_deliveries_weight=1, first_message_deliveries_decay=2, **q), False),
        (topic(first_message_deliveries_weight=1, first_message_deliveries_decay=.5, first_message_deliveries_cap=-1, **q), False),
        (topic(mesh_message_deliveries_weight=1, **q), False),
        (topic(mesh_message_deliveries_weight=-1, mesh_message_deliveries_decay=-1, **q), False),
        (topic(mesh_message_deliveries_weight=-1, mesh_message_deliveries_decay=2, **q), False),
        (topic(mesh_message_deliveries_weight=-1, mesh_message_deliveries_decay=.5, mesh_message_deliveries_cap=-1, **q), False),
        (topic(mesh_message_deliveries_weight=-1, mesh_message_deliveries_decay=.5, mesh_message_deliveries_cap=5,
               mesh_message_deliveries_threshold=-3, **q), False),
        (topic(mesh_message_deliveries_weight=-1, mesh_message_deliveries_decay=.5, mesh_message_deliveries_cap=5,
               mesh_message_deliveries_threshold=3, mesh_message_deliveries_window_ns=-1, **q), False),
        (topic(mesh_message_deliveries_weight=-1, mesh_message_deliveries_decay=.5, mesh_message_deliveries_cap=5,
               mesh_message_deliveries_threshold=3, mesh_message_deliveries_window_ns=MS,
               mesh_message_deliveries_activation_ns=MS, **q), False),
        (topic(mesh_failure_penalty_weight=1, **q), False),
        (topic(mesh_failure_penalty_weight=-1, mesh_failure_penalty_decay=-1, **q), False),
        (topic(mesh_failure_penalty_weight=-1, mesh_failure_penalty_decay=2, **q), False),
        (topic(invalid_message_deliveries_weight=1, **q), False),
        (topic(invalid_message_deliveries_weight=-1, invalid_message_deliveries_decay=-1, **q), False),
        (topic(invalid_message_deliveries_weight=-1, invalid_message_deliveries_decay=2, **q), False),
        (good, True),
    ]
    for i, (p, ok) in enumerate(tps):
        cases.append(dict(kind="topic", ref=f"score_params_test.go:51-146 #{i}", params=p, valid=ok))
    # TestPeerScoreParamsValidation, score_params_test.go:148-321 (topics validated alongside)
    base = dict(decay_interval_ns=S, decay_to_zero=0.01)
    bad_topic_inf = dict(good, topic_weight=INF, time_in_mesh_weight=NAN, first_message_deliveries_weight=INF,
                         mesh_message_deliveries_weight=-INF, mesh_message_deliveries_decay=NAN,
                         mesh_message_deliveries_cap=INF, mesh_failure_penalty_decay=NAN,
                         invalid_message_deliveries_weight=INF, invalid_message_deliveries_decay=NAN)
    pps = [
        (peer(topic_score_cap=-1, **base), [], False),
        (dict(peer(topic_score_cap=1, **base), app_specific_score_set=0), [], False),
        (peer(topic_score_cap=1, ip_colocation_factor_weight=1, **base), [], False),
        (peer(topic_score_cap=1, ip_colocation_factor_weight=-1, ip_colocation_factor_threshold=-1, **base), [], False),
        (peer(topic_score_cap=1, decay_interval_ns=MS, decay_to_zero=0.01, ip_colocation_factor_weight=-1,
              ip_colocation_factor_threshold=1), [], False),
        (peer(topic_score_cap=1, decay_interval_ns=S, decay_to_zero=-1, ip_colocation_factor_weight=-1,
              ip_colocation_factor_threshold=1), [], False),
        (peer(topic_score_cap=1, decay_interval_ns=S, decay_to_zero=2, ip_colocation_factor_weight=-1,
              ip_colocation_factor_threshold=1), [], False),
        (peer(behaviour_penalty_weight=1, **base), [], False),
        (peer(behaviour_penalty_weight=-1, **base), [], False),
        (peer(behaviour_penalty_weight=-1, behaviour_penalty_decay=2, **base), [], False),
        (peer(ip_colocation_factor_weight=-1, ip_colocation_factor_threshold=1, behaviour_penalty_weight=-1,
              behaviour_penalty_decay=0.999, **base), [], True),
        (peer(topic_score_cap=1, ip_colocation_factor_weight=-1, ip_colocation_factor_threshold=1,
              behaviour_penalty_weight=-1, behaviour_penalty_decay=0.999, **base), [], True),
        (peer(topic_score_cap=1, ip_colocation_factor_weight=-1, ip_colocation_factor_threshold=1, **base), [good], True),
        (peer(topic_score_cap=1, ip_colocation_factor_weight=-1, ip_colocation_factor_threshold=1, **base),
         [dict(good, topic_weight=-1)], False),
        (peer(decay_interval_ns=S, decay_to_zero=INF, ip_colocation_factor_weight=-INF, ip_colocation_factor_threshold=1,
              behaviour_penalty_weight=INF, behaviour_penalty_decay=NAN), [], False),
        (peer(topic_score_cap=1, ip_colocation_factor_weight=-1, ip_colocation_factor_threshold=1, **base),
         [bad_topic_inf], False),
    ]
    for i, (p, tl, ok) in enumerate(pps):
        cases.append(dict(kind="peer", ref=f"score_params_test.go:148-321 #{i}", params=p, topics=tl, valid=ok))
    return cases


def decay_cases():
    # TestScoreParameterDecay, score_params_test.go:323-328
    return [dict(ref="score_params_test.go:323-328", decay_ns=HOUR, expected=0.9987216039048303)]


def promise_cases():
    """gossip_tracer_test.go: the gossipTracer's promise bookkeeping.

    Peers A, B, C are the observer's pairs 0, 1, 2; mids are the handles
    1 << 32 | i of 100 messages.  Times are offsets from the moment of the
    AddPromise calls.  `followup_ns` is the tracer's followUpTime; a
    GetBrokenPromises step lists the per-peer counts the test asserts (an
    empty dict for "expected no broken promises", i.e. a nil map)."""
    mids = [(1 << 32) | i for i in range(100)]
    broken = dict(
        name="TestBrokenPromises", ref="gossip_tracer_test.go:12-57",
        # gt.followUpTime = 100 ms; the sleep is GossipSubIWantFollowupTime (3 s) + 10 ms
        followup_ns=100 * MS, peers=["A", "B", "C"], mids=mids,
        steps=[
            dict(op="add", peer="A"), dict(op="add", peer="B"), dict(op="add", peer="C"),
            dict(op="broken", at_ns=0, expect={}),
            dict(op="throttle", peer="C"),
            dict(op="broken", at_ns=3 * S + 10 * MS, expect={"A": 1, "B": 1}),
        ],
    )
    none = dict(
        name="TestNoBrokenPromises", ref="gossip_tracer_test.go:59-97",
        # newGossipTracer() without Start: followUpTime is the zero Duration, the
        # promises expire at once; DeliverMessage fulfils all of them first
        followup_ns=0, peers=["A", "B"], mids=mids,
        steps=[
            dict(op="add", peer="A"), dict(op="add", peer="B"),
            dict(op="deliver_all"),
            dict(op="broken", at_ns=110 * MS, expect={}),
        ],
    )
    return [broken, none]


def main():
    with open(os.path.join(OUT, "promise_kat.json"), "w") as f:
        json.dump(promise_cases(), f, indent=1)
    sc = scenarios()
    with open(os.path.join(OUT, "score_kat.json"), "w") as f:
        json.dump(_enc(sc), f, indent=0)
    with open(os.path.join(OUT, "params_validation.json"), "w") as f:
        json.dump(_enc(dict(validation=validation_cases(), decay=decay_cases())), f, indent=1)
    print(f"wrote {len(sc)} score scenarios")


if __name__ == "__main__":
    main()
