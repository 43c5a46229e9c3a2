"""The oracle restates gossipsub's graylist gate on forwarded messages:
TestGossipsubAttackInvalidMessageSpam (gossipsub_spam_test.go:615-763), see
tests/spam_cases.py."""
import oracle as orc
import spam_cases as sc


def test_invalid_message_spam_stops_at_graylist():
    o = orc.Oracle(1)
    rows = sc.run(o)
    sc.check(rows)
    # the legit node then prunes the negative-score attacker at its heartbeat
    # (gossipsub.go:1362-1368), the reference test's PRUNE assertion
    sc.check_prune(sc.heartbeat(o))
