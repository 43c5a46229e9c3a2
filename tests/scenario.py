"""Drives a known-answer scenario (tests/golden/score_kat.json) through a backend.

A backend is anything with the gsx.Engine method set: the HIP engine through
the C ABI, or the CPU oracle (oracle/oracle.py).  The scenario's single router
is observer node 0; its peers are nodes 1..K, pair i standing for peers[i].
"""
from __future__ import annotations

import ipaddress
import json
import math
import os

import numpy as np

from gsx import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T0 = 1_700_000_000 * abi.SECOND
TIME_CACHE_DURATION = 120 * abi.SECOND  # pubsub.go:30


def _dec(x):
    if isinstance(x, str) and x in ("inf", "-inf", "nan"):
        return float(x)
    if isinstance(x, dict):
        return {k: _dec(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_dec(v) for v in x]
    return x


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return _dec(json.load(f))


def same(a: float, b: float) -> bool:
    """Bit-exact float equality (Go's `!=`), with NaN == NaN."""
    return a == b or (math.isnan(a) and math.isnan(b))


def run_scenario(sc, make_backend):
    """Returns a list of mismatch strings (empty == pass)."""
    peers = sc["peers"]
    K = len(peers)
    pidx = {p: i for i, p in enumerate(peers)}
    topics = list(sc["topic_params"].keys()) or ["mytopic"]
    tidx = {t: i for i, t in enumerate(topics)}
    if "mytopic" not in tidx:
        tidx["mytopic"] = len(topics)
        topics.append("mytopic")

    ip_ids = {}
    node_ips = np.full((K + 1, 2), abi.GSX_NO_IP, dtype=np.uint32)
    for p, lst in sc.get("ips", {}).items():
        for k, ip in enumerate(lst):
            node_ips[1 + pidx[p], k] = ip_ids.setdefault(ip, len(ip_ids))

    be = make_backend(len(topics))
    be.set_peer_params(abi.PeerScoreParams(**sc["peer_params"]))
    for t, tp in sc["topic_params"].items():
        be.set_topic_params(tidx[t], abi.TopicScoreParams(**tp))
    row_ptr = np.array([0] + [K] * (K + 1), dtype=np.int64)
    col = np.arange(1, K + 1, dtype=np.int32)
    be.load_overlay(row_ptr, col, None, node_ips)
    if "whitelist_cidr" in sc:
        net = ipaddress.ip_network(sc["whitelist_cidr"])
        be.set_ip_whitelist([i for ip, i in ip_ids.items() if ipaddress.ip_address(ip) in net])
    app = np.zeros(K, dtype=np.float64)
    for p, v in sc.get("app", {}).items():
        app[pidx[p]] = v
    be.set_app_scores(app)

    now = T0
    bad = []

    def ev(kind, p, topic=0, arg=0):
        be.apply_events(np.array([(kind, topic, pidx[p], now, arg)], dtype=abi.event_dtype()))

    for i, st in enumerate(sc["steps"]):
        op = st[0]
        if op == "add_peer":
            ev(abi.EV_ADD_PEER, st[1])
        elif op == "remove_peer":
            ev(abi.EV_REMOVE_PEER, st[1])
        elif op == "graft":
            ev(abi.EV_GRAFT, st[1], tidx[st[2]])
        elif op == "prune":
            ev(abi.EV_PRUNE, st[1], tidx[st[2]])
        elif op == "penalty":
            ev(abi.EV_PENALTY, st[1], 0, st[2])
        elif op == "validate":
            be.trace_validate(pidx[st[1]], st[2], tidx[st[3]], now)
        elif op == "deliver":
            be.trace_deliver(pidx[st[1]], st[2], tidx[st[3]], now)
        elif op == "duplicate":
            be.trace_duplicate(pidx[st[1]], st[2], tidx[st[3]], now)
        elif op == "reject":
            be.trace_reject(pidx[st[1]], st[2], tidx[st[3]], abi.REJECT_REASONS[st[4]], now)
        elif op == "advance":
            now += int(st[1])
        elif op == "refresh":
            be.refresh(now)
        elif op == "gc_expire_all":
            now += TIME_CACHE_DURATION + abi.MILLISECOND
            be.gc_deliveries(now)
            if be.num_delivery_records() != 0:
                bad.append(f"step {i}: gc left {be.num_delivery_records()} records")
        elif op == "set_app":
            app[pidx[st[1]]] = st[2]
            be.set_app_scores(app)
        elif op == "set_topic_params":
            be.set_topic_params(tidx[st[1]], abi.TopicScoreParams(**st[2]))
        elif op in ("expect_score", "expect_score_ge"):
            got = be.score(pidx[st[1]])
            want = float(st[2])
            ok = same(got, want) if op == "expect_score" else got >= want
            if not ok:
                bad.append(f"step {i} {op} {st[1]}: got {got!r} want {want!r}")
        elif op == "expect_counter":
            stt = be.export_state()
            got = float(stt[st[3]][tidx[st[2]] * K + pidx[st[1]]])
            if not same(got, float(st[4])):
                bad.append(f"step {i} counter {st[3]} {st[1]}: got {got!r} want {st[4]!r}")
        else:
            raise ValueError(op)
    return bad
