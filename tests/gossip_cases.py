"""Gossip exchange scenarios (gsx.h heartbeat step (D): handleIHave /
handleIWant, gossipsub.go:615-716; promises, gossip_tracer.go:48-153), driven
identically through any backend (the engine or the oracle)."""
from __future__ import annotations

import numpy as np

import heartbeat_cases as hc
import propagation_cases as pc
from gsx import abi

S = abi.SECOND
MS = abi.MILLISECOND


def params(**kw):
    """DefaultGossipSubParams with the exchange on, and overrides."""
    from oracle import default_gossipsub_params

    gp = default_gossipsub_params()
    gp.gossip_exchange = 1
    for k, v in kw.items():
        setattr(gp, k, v)
    return gp


def exchange_run(be, n=300, d=6, T=2, seed=5, ticks=8, hops=2, msgs=24, invalid=0.0, exchange_from=0, prefill=0,
                 runner=None, credit=None, window_ms=None, latency_ms=5, delay_ms=0.0, **gp_kw):
    """pc.setup's random mesh; every round: a heartbeat (with the exchange),
    then a gossipsub batch that travels only `hops` hops (so most nodes miss
    it and learn of it by IHAVE), then a refresh.  Rounds before
    `exchange_from` only emit IHAVEs; `prefill` promises per pair are made
    before the first round (the engine's per-pair slots fill and grow).
    runner: a gsx.shard.MessageParallel over `be` (its propagate and
    heartbeat replace the backend's); credit: the batches' credit mode;
    window_ms: MeshMessageDeliveriesWindow (default pc.setup's 25 ms: every
    old copy outside by the next heartbeat); latency_ms / delay_ms: the
    batches' hop latency and validation delay (an old copy was validated at
    the batch's now + hop * (latency + delay), or at the heartbeat that
    recovered it).
    Returns per-tick counters
    and snapshots (records, backoff, scores, IHAVEs) plus every node's cached
    ids after the last round."""
    ov = pc.overlay(n, d, seed)
    pc.setup(be, ov, T, seed, mesh_degree=6)
    if window_ms is not None:
        from gsx import synth

        for t in range(T):
            tp = synth.spam_test_topic_params()
            tp.mesh_message_deliveries_window_ns = int(window_ms * MS)
            be.set_topic_params(t, tp)
    for q in range(ov.n_pairs if prefill else 0):  # promises no exchange fulfils, expiring late
        for j in range(prefill):
            be.promise_add(q, [(0xFFFF << 32) | (q * prefill + j)], hc.T0 + 10**6 * S)
    outs, snaps = [], []
    for k in range(ticks):
        if k <= exchange_from:  # no exchange before round exchange_from
            gp = params(**gp_kw)
            if k < exchange_from:
                gp.gossip_exchange = 0
            be.set_gossipsub_params(gp)
        now = hc.T0 + (3 + k) * S
        if runner is None:
            outs.append(be.heartbeat(1 + k, now, seed * 31 + 7).as_dict())
        else:
            outs.append(runner.heartbeat(1 + k, now, seed * 31 + 7)[0])
        snaps.append(hc.snapshot(be))
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, max_hops=hops, latency_ms=latency_ms, seed=seed + k,
                        delay_ms=delay_ms)
        if credit is not None:
            cfg.credit_scores = credit
        cfg.now_ns = now + 100 * MS
        ms = pc.messages(n, msgs, seed + 1000 * k, invalid=invalid)
        (runner or be).propagate(ms, cfg)
        be.refresh(now + 500 * MS)
    cached = [be.mcache_ids(v, abi.GSX_ANY_TOPIC, 5) for v in range(n)]
    return ov, outs, snaps, cached
