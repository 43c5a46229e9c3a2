"""The oracle's multi-threaded refresh+score (bench.py's OpenMP CPU baseline)
equals the serial refreshScores() + score() bit for bit."""
import numpy as np

import oracle as orc
from gsx import abi, synth


def test_parallel_refresh_equals_serial():
    n, T = 3000, 3
    ov = synth.connect_some_overlay(n, d=6, sybil_frac=0.2, sybils_per_ip=50)
    now = 1_700_000_000 * abi.SECOND
    st = synth.synthetic_state(ov, T, now, p_disconnected=0.1, p_absent=0.05)
    res = []
    for threads in (None, 4):
        o = orc.Oracle(T)
        o.set_peer_params(synth.bench_peer_params())
        for t in range(T):
            o.set_topic_params(t, synth.spam_test_topic_params())
        o.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
        o.import_state(st)
        o.set_app_scores(np.linspace(-3, 3, ov.n_pairs))
        for k in range(3):
            if threads is None:
                o.refresh(now + (k + 1) * abi.SECOND)
                sc = o.scores()
            else:
                sc = o.refresh_scores_parallel(now + (k + 1) * abi.SECOND, threads)
        ex = o.export_state()
        res.append((sc, ex))
    (a, ea), (b, eb) = res
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))
    for f in abi.STATE_FIELDS:
        assert np.array_equal(ea[f].view(np.uint8), eb[f].view(np.uint8)), f
