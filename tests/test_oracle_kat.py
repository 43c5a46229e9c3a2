"""The CPU oracle against the reference's own known answers (CPU only).

Pins oracle/gsx_oracle.c to score_test.go / score_params_test.go through the
fixtures in tests/golden/ (see make_golden.py for how each was taken).
"""
import math

import pytest

import oracle as orc
from gsx import abi
from scenario import load_json, run_scenario

KAT = load_json("score_kat.json")
VAL = load_json("params_validation.json")


@pytest.mark.parametrize("sc", KAT, ids=[s["name"] for s in KAT])
def test_oracle_score_kat(sc):
    bad = run_scenario(sc, lambda T: orc.Oracle(T))
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("case", VAL["validation"], ids=[c["ref"] for c in VAL["validation"]])
def test_oracle_params_validation(case):
    if case["kind"] == "thresholds":
        ok = orc.validate_thresholds(abi.Thresholds(**case["params"])) == 0
    elif case["kind"] == "topic":
        ok = orc.validate_topic_params(abi.TopicScoreParams(**case["params"])) == 0
    else:
        ok = orc.validate_peer_params(abi.PeerScoreParams(**case["params"])) == 0
        ok = ok and all(orc.validate_topic_params(abi.TopicScoreParams(**t)) == 0 for t in case["topics"])
    assert ok == case["valid"]


def test_oracle_score_parameter_decay():
    for c in VAL["decay"]:
        assert orc.score_parameter_decay(c["decay_ns"]) == c["expected"]
    # ScoreParameterDecayWithBase uses integer Duration division (score_params.go:285)
    assert orc.score_parameter_decay_with_base(1500 * abi.MILLISECOND, abi.SECOND, 0.01) == math.pow(0.01, 1.0)
