"""Trace export from GPU results (gsx/trace.py): the GRAFT /
PRUNE stream of a heartbeat and the DELIVER_MESSAGE / REJECT_MESSAGE / DUPLICATE_MESSAGE stream of a propagation
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


@pytest.mark.parametrize("case", test_trace_cases := __import__("test_trace").CASES)
def test_delivery_trace_gpu_equals_oracle(gpu_ok, case):
    """PUBLISH / DELIVER / REJECT / DUPLICATE streams (gsx_prop_duplicates for the
    DUPLICATE events) byte-equal to the oracle's, for every router, graylisted
    senders and a hop limit."""
    invalid, delay_ms, router, gray, max_hops = case
    T = len(tc.TOPICS)
    kw = dict(invalid=invalid, delay_ms=delay_ms, router=router, gray=gray, max_hops=max_hops)
    g = tc.delivery_stream(gsx.Engine(T), **kw)
    w = tc.delivery_stream(orc.Oracle(T), **kw)
    assert np.array_equal(g[5], w[5])
    assert g[4].duplicates == w[4].duplicates == int(sum(bin(int(x)).count("1") for x in g[5].ravel()))
    assert len(g[0]) > 0 and g[0] == w[0]
