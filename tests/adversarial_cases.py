"""BASELINE.md cfg5 at test size: sybils in IP groups attacking victim nodes
(P6, score.go:337-381) and carrying invalid-message counters (P4,
score.go:305-308), loaded identically into any backend."""
from __future__ import annotations

import numpy as np

from gsx import abi, synth

S = abi.SECOND
T0 = 1_700_000_000 * S
TH = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                    accept_px_threshold=0, opportunistic_graft_threshold=0)


def setup(be, n, seed=5, sybil_frac=0.2, sybils_per_ip=50, victims=6):
    ov = synth.adversarial_overlay(n, seed=seed, sybil_frac=sybil_frac, sybils_per_ip=sybils_per_ip, victims=victims)
    be.set_peer_params(synth.bench_peer_params())
    be.set_topic_params(0, synth.spam_test_topic_params())
    be.set_thresholds(TH)
    be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    st = synth.synthetic_state(ov, 1, T0, seed=seed)
    be.import_state(st)
    be.set_app_scores(np.zeros(ov.n_pairs))
    be.refresh(T0 + S)
    return ov


def sybil_pairs(ov):
    return ov.sybil[ov.col]


def victim_pairs(ov, min_colocated=10):
    """Pairs whose peer shares its IP with at least min_colocated - 1 other
    peers of the same observer (a sybil group attacking that observer)."""
    obs = ov.pair_observer()
    ip = ov.node_ips[ov.col, 0].astype(np.int64)
    key = obs * (1 << 32) + ip
    u, inv, c = np.unique(key, return_inverse=True, return_counts=True)
    return c[inv] >= min_colocated
