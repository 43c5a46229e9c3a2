"""The oracle's gossipTracer against the reference's promise tests
(gossip_tracer_test.go:12-97, fixtures in tests/golden/promise_kat.json)."""
import pytest

import oracle as orc
import promise_cases as pc


@pytest.mark.parametrize("case", pc.load(), ids=lambda c: c["name"])
def test_promise_kat_oracle(case):
    assert pc.run(orc.Oracle(1), case) == []


def test_promise_table_is_unbounded():
    """AddPromise never refuses (gossip_tracer.go:59-74): 1000 promises on one pair."""
    o = orc.Oracle(1)
    row_ptr, col = pc.star(2)
    from gsx import synth

    o.set_peer_params(synth.bench_peer_params())
    o.load_overlay(row_ptr, col)
    for k in range(1000):
        o.promise_add(0, [k], pc.T0 + k)
    o.promise_add(0, [5], pc.T0)  # an existing (pair, message) promise is kept, not re-added
    assert o.promise_count() == 1000
    cnt, tot = o.promise_broken(pc.T0 + 500)
    assert tot == 500 and cnt[0] == 500 and o.promise_count() == 500
    o.promise_fulfill(0, 700)
    assert o.promise_count() == 499
    o.promise_throttle(0)
    assert o.promise_count() == 0


def test_promise_expiry_zero_is_refused():
    """Expiry 0 is the engine's free-slot mark (gsx.h): both backends refuse it
    instead of storing a promise one of them would not see."""
    o = orc.Oracle(1)
    row_ptr, col = pc.star(2)
    from gsx import synth

    o.set_peer_params(synth.bench_peer_params())
    o.load_overlay(row_ptr, col)
    with pytest.raises(Exception):
        o.promise_add(0, [1], 0)
    assert o.promise_count() == 0
