"""Shared trace-export cases (gsx/trace.py): a heartbeat and a propagation run on
any backend (gsx.Engine or the oracle), turned into delimited TraceEvent streams."""
import numpy as np

import heartbeat_cases as hc
import propagation_cases as pc
from gsx import abi
from gsx import trace as tr

TOPICS = ["topic-a", "topic-b"]


def heartbeat_stream(be, n=400, d=6, seed=11):
    """One traced heartbeat after pc.setup's random mesh: (stream, counters, in-mesh
    count before, tracer words)."""
    T = len(TOPICS)
    ov = pc.overlay(n, d, seed)
    pc.setup(be, ov, T, seed, mesh_degree=6)
    before = be.export_state()["rec_flags"].copy()
    be.hb_set_tracing(True)
    out = be.heartbeat(1, hc.T0 + 3 * hc.S, seed * 31 + 7).as_dict()
    words = be.hb_trace_words()
    ev = list(tr.mesh_trace(words, ov.row_ptr, ov.col, TOPICS, hc.T0 + 3 * hc.S))
    links_before = int(np.count_nonzero(before & abi.GSX_REC_IN_MESH))
    return tr.write_delimited(ev), out, links_before, words


def delivery_stream(be, n=500, m=40, seed=7, invalid=0.0, delay_ms=0.0):
    """One gossipsub propagation with first-deliverer rows: (stream, hop, first_from, msgs)."""
    T = len(TOPICS)
    ov = pc.overlay(n, 6, seed)
    pc.setup(be, ov, T, seed)
    ms = pc.messages(n, m, seed, invalid=invalid)
    cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=1, latency_ms=10, delay_ms=delay_ms)
    _, hop, frm = be.propagate(ms, cfg, want_results=True)
    ev = tr.delivery_trace(hop, frm, ms, TOPICS[1], int(cfg.now_ns), int(cfg.hop_latency_ns),
                          validation_delay_ns=int(cfg.validation_delay_ns))
    return tr.write_delimited(ev), hop, frm, ms
