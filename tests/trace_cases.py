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


def delivery_stream(be, n=500, m=40, seed=7, invalid=0.0, delay_ms=0.0, router=abi.GSX_ROUTER_GOSSIPSUB,
                    gray=False, max_hops=40):
    """One propagation with first-deliverer rows and duplicate rows: (stream, hop,
    first_from, msgs, out, dup_rows).  ``gray``: a fifth of the pairs score below
    the graylist threshold (their copies are dropped, not traced)."""
    T = len(TOPICS)
    ov = pc.overlay(n, 6, seed)
    pc.setup(be, ov, T, seed)
    if gray:
        app = np.zeros(ov.n_pairs)
        app[np.random.default_rng(seed).random(ov.n_pairs) < 0.2] = -1e6
        be.set_app_scores(app)
    ms = pc.messages(n, m, seed, invalid=invalid)
    cfg = pc.config(router, topic=1, latency_ms=10, delay_ms=delay_ms, max_hops=max_hops, size=40)
    if hasattr(be, "set_dup_tracking"):  # the oracle records duplicates on request
        be.set_dup_tracking(True)
    out, hop, frm = be.propagate(ms, cfg, want_results=True)
    dup = be.prop_duplicates(len(ms))
    ev = tr.delivery_trace(hop, frm, ms, TOPICS[1], int(cfg.now_ns), int(cfg.hop_latency_ns),
                           validation_delay_ns=int(cfg.validation_delay_ns), dup_rows=dup, row_ptr=ov.row_ptr,
                           col=ov.col)
    return tr.write_delimited(ev), hop, frm, ms, out, dup
