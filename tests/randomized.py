"""Seeded random call sequences over the whole scoring interface, replayed on
any backend (HIP engine or CPU oracle) so their results can be compared
bit-for-bit.  Covers every event kind, every tracer call and reject reason,
retention/expiry, IP colocation with a whitelist, app scores, topic-param
resets with recap, an unscored topic, and delivery-record gc."""
from __future__ import annotations

import numpy as np

from gsx import abi, synth

S = abi.SECOND
MS = abi.MILLISECOND
T0 = 1_700_000_000 * S

REASONS = list(abi.REJECT_REASONS.values())


def scenario_params(n_topics):
    pp = abi.PeerScoreParams(
        topic_score_cap=30.0,
        app_specific_weight=0.75,
        app_specific_score_set=1,
        ip_colocation_factor_threshold=1,
        ip_colocation_factor_weight=-3.5,
        behaviour_penalty_weight=-2.0,
        behaviour_penalty_threshold=1.5,
        behaviour_penalty_decay=0.9,
        decay_interval_ns=S,
        decay_to_zero=0.01,
        retain_score_ns=3 * S,
    )
    tps = {}
    for t in range(n_topics - 1):  # the last topic stays unscored
        tp = synth.spam_test_topic_params()
        tp.topic_weight = 0.25 + 0.5 * t
        tp.time_in_mesh_quantum_ns = (t + 1) * 700 * MS
        tp.time_in_mesh_cap = 5.0 + t
        tp.mesh_message_deliveries_activation_ns = (2 + t) * S
        tp.mesh_message_deliveries_window_ns = 400 * MS
        tp.mesh_message_deliveries_threshold = 4.0 + t
        tp.mesh_message_deliveries_cap = 12.0
        tp.first_message_deliveries_cap = 9.0 + t
        tp.first_message_deliveries_decay = 0.8
        tp.mesh_message_deliveries_decay = 0.85
        tp.mesh_failure_penalty_decay = 0.9
        tp.invalid_message_deliveries_decay = 0.95
        tps[t] = tp
    return pp, tps


def small_overlay(n, d, seed, n_ip_pool):
    ov = synth.connect_some_overlay(n, d=d, seed=seed)
    rng = np.random.default_rng(seed)
    ips = np.full((n, 2), abi.GSX_NO_IP, dtype=np.uint32)
    ips[:, 0] = rng.integers(0, n_ip_pool, n)
    two = rng.random(n) < 0.3
    ips[two, 1] = rng.integers(0, n_ip_pool, int(two.sum()))
    same = rng.random(n) < 0.05  # a duplicated IP in the list (counted twice, tracked once)
    ips[same, 1] = ips[same, 0]
    ov.node_ips = ips
    return ov


def n_ip_pool(ov):
    ips = ov.node_ips[ov.node_ips != abi.GSX_NO_IP]
    return int(ips.max()) + 1 if len(ips) else 8


def make_ops(ov, n_topics, seed, n_steps=400):
    rng = np.random.default_rng(seed + 1)
    E = ov.n_pairs
    obs_of = ov.pair_observer()
    rows = [np.arange(ov.row_ptr[i], ov.row_ptr[i + 1]) for i in range(ov.n)]
    now = T0
    ops = []
    # connect most pairs first
    first = np.nonzero(rng.random(E) < 0.9)[0]
    ops.append(("events", [(abi.EV_ADD_PEER, 0, int(p), now, 0) for p in first]))
    grafts = first[rng.random(len(first)) < 0.6]
    ops.append(("events", [(abi.EV_GRAFT, int(rng.integers(0, n_topics)), int(p), now, 0) for p in grafts]))
    ops.append(("check",))
    msg = 0
    for step in range(n_steps):
        now += int(rng.integers(0, 600)) * MS
        r = rng.random()
        if r < 0.35:
            evs = []
            for _ in range(int(rng.integers(1, 40))):
                kind = int(rng.integers(1, 9))
                p = int(rng.integers(0, E))
                t = int(rng.integers(0, n_topics))
                arg = int(rng.integers(1, 4)) if kind == abi.EV_PENALTY else 0
                if kind == abi.EV_REMOVE_PEER and rng.random() < 0.5:
                    kind = abi.EV_ADD_PEER
                evs.append((kind, t, p, now, arg))
            ops.append(("events", evs))
        elif r < 0.75:
            # a message seen by one observer from several of its neighbours
            o = int(rng.integers(0, ov.n))
            if len(rows[o]) == 0:
                continue
            msg += 1
            m = msg if rng.random() < 0.8 else int(rng.integers(1, msg + 1))
            t = int(rng.integers(0, n_topics))
            nb = rng.permutation(rows[o])[: int(rng.integers(1, 5))]
            seq = []
            seq.append(("validate", int(nb[0]), m, t, now))
            for q in nb[1:]:
                if rng.random() < 0.5:
                    seq.append(("duplicate", int(q), m, t, now))
            c = rng.random()
            if c < 0.6:
                seq.append(("deliver", int(nb[0]), m, t, now))
            else:
                seq.append(("reject", int(nb[0]), m, t, int(rng.choice(REASONS)), now))
            later = now + int(rng.integers(0, 800)) * MS
            for q in nb[1:]:
                if rng.random() < 0.6:
                    seq.append(("duplicate", int(q), m, t, later))
            if rng.random() < 0.2:
                seq.append(("duplicate", int(nb[0]), m, t, later))
            ops.append(("trace", seq))
        elif r < 0.85:
            ops.append(("refresh", now))
        elif r < 0.88:
            app = rng.normal(0, 3, E)
            app[rng.random(E) < 0.5] = 0.0
            ops.append(("app", app))
        elif r < 0.90:
            t = int(rng.integers(0, n_topics - 1))
            _, tps = scenario_params(n_topics)
            tp = tps[t]
            tp.first_message_deliveries_cap = float(rng.integers(3, 12))
            tp.mesh_message_deliveries_cap = float(rng.integers(3, 12))
            tp.invalid_message_deliveries_weight = -float(rng.integers(1, 50))
            ops.append(("topic_params", t, tp))
        elif r < 0.92:
            ops.append(("gc", now + int(rng.integers(0, 200)) * S))
        elif r < 0.95:  # refreshIPs / AddPeer on new addresses: some pairs' IP lists change
            k = int(rng.integers(1, 12))
            pairs = rng.integers(0, E, k)
            ips = rng.integers(0, n_ip_pool(ov) + 4, (k, 2)).astype(np.uint32)
            ips[rng.random((k, 2)) < 0.25] = abi.GSX_NO_IP
            dup = rng.random(k) < 0.1
            ips[dup, 1] = ips[dup, 0]
            ops.append(("ips", pairs, ips))
        else:
            ops.append(("check",))
        if step % 50 == 49:
            ops.append(("refresh", now))
            ops.append(("check",))
    ops.append(("refresh", now + S))
    ops.append(("check",))
    return ops


def replay(be, ov, n_topics, ops, whitelist=(3,)):
    pp, tps = scenario_params(n_topics)
    be.set_peer_params(pp)
    for t, tp in tps.items():
        be.set_topic_params(t, tp)
    be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    be.set_ip_whitelist(list(whitelist))
    snaps = []
    for op in ops:
        k = op[0]
        if k == "events":
            be.apply_events(np.array(op[1], dtype=abi.event_dtype()))
        elif k == "trace":
            for c in op[1]:
                getattr(be, "trace_" + c[0])(*c[1:])
        elif k == "refresh":
            be.refresh(op[1])
        elif k == "app":
            be.set_app_scores(op[1])
        elif k == "topic_params":
            be.set_topic_params(op[1], op[2])
        elif k == "gc":
            be.gc_deliveries(op[1])
        elif k == "ips":
            be.set_pair_ips(op[1], op[2])
        elif k == "check":
            snaps.append((be.scores(), be.export_state(), be.num_delivery_records()))
    return snaps


def interleaved_score_calls(be, ov, n_topics, ops, seed, per_call=2, many=False):
    """Replay ``ops`` one call at a time (every event and tracer call on its
    own), asking Score() of a few random pairs after each: what a router does
    between RPCs (gossipsub.go:589 AcceptFrom, :960-989 Publish); with
    `many` the pairs of one ask go through one score_many call
    (gsx_score_many).  Returns the scores asked, in order."""
    rng = np.random.default_rng(seed + 99)
    pp, tps = scenario_params(n_topics)
    be.set_peer_params(pp)
    for t, tp in tps.items():
        be.set_topic_params(t, tp)
    be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    be.set_ip_whitelist([3])
    E = ov.n_pairs
    out = []

    def ask():
        ps = rng.integers(0, E, per_call)
        if many:
            out.extend(float(x) for x in be.score_many(ps.astype(np.uint64)))
            return
        for p in ps.tolist():
            out.append(be.score(int(p)))

    for op in ops:
        k = op[0]
        if k == "events":
            if len(op[1]) >= 50:  # the initial AddPeer / Graft batches go in one call
                be.apply_events(np.array(op[1], dtype=abi.event_dtype()))
                ask()
                continue
            for ev in op[1]:
                be.apply_events(np.array([ev], dtype=abi.event_dtype()))
                ask()
        elif k == "trace":
            for c in op[1]:
                getattr(be, "trace_" + c[0])(*c[1:])
                ask()
        elif k == "refresh":
            be.refresh(op[1])
            ask()
        elif k == "app":
            be.set_app_scores(op[1])
            ask()
        elif k == "topic_params":
            be.set_topic_params(op[1], op[2])
            ask()
        elif k == "ips":
            be.set_pair_ips(op[1], op[2])
            ask()
    return np.array(out)
