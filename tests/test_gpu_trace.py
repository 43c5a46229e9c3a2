"""Trace export from GPU results (gsx/trace.py): the GRAFT /
PRUNE stream of a heartbeat and the DELIVER_MESSAGE / REJECT_MESSAGE stream of a propagation
are byte-identical to the streams built from the oracle's results."""
import numpy as np
import pytest

import gsx
import oracle as orc
import trace_cases as tc

pytestmark = pytest.mark.gpu


def test_heartbeat_trace_gpu_equals_oracle(gpu_ok):
    T = len(tc.TOPICS)
    g = tc.heartbeat_stream(gsx.Engine(T))
    w = tc.heartbeat_stream(orc.Oracle(T))
    assert g[1] == w[1] and g[2] == w[2]
    for a, b in zip(g[3], w[3]):
        assert np.array_equal(a, b)
    assert len(g[0]) > 0 and g[0] == w[0]


@pytest.mark.parametrize("invalid,delay_ms", [(0.0, 0.0), (0.3, 0.0), (0.3, 4.0)])
def test_delivery_trace_gpu_equals_oracle(gpu_ok, invalid, delay_ms):
    T = len(tc.TOPICS)
    g = tc.delivery_stream(gsx.Engine(T), invalid=invalid, delay_ms=delay_ms)[0]
    w = tc.delivery_stream(orc.Oracle(T), invalid=invalid, delay_ms=delay_ms)[0]
    assert len(g) > 0 and g == w
