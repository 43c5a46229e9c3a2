"""The reference's gossipTracer tests (gossip_tracer_test.go) restated as
fixtures (tests/golden/promise_kat.json) and driven through a backend's
promise calls (gsx_promise_*, gossip_tracer.go:48-185)."""
from __future__ import annotations

import json
import os

import numpy as np

T0 = 1_700_000_000 * 1_000_000_000
HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with open(os.path.join(HERE, "golden", "promise_kat.json")) as f:
        return json.load(f)


def star(n_peers):
    """Observer 0 connected to peers 1..n (pairs 0..n-1 are A, B, C, ...)."""
    row_ptr = np.array([0, n_peers] + [n_peers + i + 1 for i in range(n_peers)], dtype=np.int64)
    col = np.array(list(range(1, n_peers + 1)) + [0] * n_peers, dtype=np.int32)
    return row_ptr, col


def run(be, case):
    """Runs one fixture; returns the list of failures (empty when it passes)."""
    from gsx import synth

    peers = case["peers"]
    row_ptr, col = star(len(peers))
    be.set_peer_params(synth.bench_peer_params())
    be.load_overlay(row_ptr, col)
    mids = np.array(case["mids"], dtype=np.uint64)
    pair = {p: i for i, p in enumerate(peers)}
    bad = []
    for i, st in enumerate(case["steps"]):
        op = st["op"]
        if op == "add":  # AddPromise at T0, expiring followUpTime later
            be.promise_add(pair[st["peer"]], mids, T0 + case["followup_ns"], seed=i)
        elif op == "throttle":
            be.promise_throttle(pair[st["peer"]])
        elif op == "deliver_all":  # DeliverMessage of every message: fulfillPromise
            for m in mids:
                be.promise_fulfill(0, int(m))
        elif op == "broken":
            cnt, tot = be.promise_broken(T0 + st["at_ns"])
            got = {p: int(cnt[pair[p]]) for p in peers if cnt[pair[p]]}
            if got != st["expect"]:
                bad.append(f"{case['name']} step {i}: broken {got}, expected {st['expect']}")
            if tot != sum(st["expect"].values()):
                bad.append(f"{case['name']} step {i}: total {tot}")
    return bad
