"""BASELINE cfg1 (TestSparseGossipsub, gossipsub_test.go:43-82) on the oracle:
the completeness the reference asserts (tests/sparse_cases.py)."""
import oracle as orc
import sparse_cases as sc


def test_sparse_gossipsub_delivers_everything():
    assert sc.connected(sc.overlay())
    hbs, res = sc.run(orc.Oracle(1))
    sc.check(hbs, res)
