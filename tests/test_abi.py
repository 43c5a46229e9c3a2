"""The C-ABI library: loads, exports every entry point of include/gsx.h, and its
host-only helpers (validate(), ScoreParameterDecay) match the reference's
known answers.  No device work here (CPU suite)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import gsx
from gsx import abi
from scenario import load_json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsx.h")
LIB = os.path.join(ROOT, "go-libp2p-pubsub_amd", "gsx", "libgsx.so")
VAL = load_json("params_validation.json")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gsx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_abi():
    fns = declared_functions()
    assert len(fns) >= 30
    assert set(fns) == set(abi.SIGNATURES), set(fns) ^ set(abi.SIGNATURES)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gsx_[a-z0-9_]+)$", out, flags=re.M))
    missing = set(declared_functions()) - exported
    assert not missing, missing


def test_library_is_gfx950_code_object():
    # the embedded offload bundle names its target: hipv4-amdgcn-amd-amdhsa--gfx950
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"--gfx942" not in data and b"--gfx90a" not in data


def test_load_and_abi_version():
    lib = gsx.load_library()
    assert lib.gsx_abi_version() == 5


def test_create_fails_loudly_without_gfx950():
    lib = gsx.load_library()
    h = C.c_void_p()
    cfg = abi.Config(n_topics=1, device=0)
    rc = lib.gsx_create(C.byref(cfg), C.byref(h))
    if rc == 0:  # a GPU box: creation works, nothing else to check here
        lib.gsx_destroy(h)
    else:
        assert rc == abi.GSX_ENODEV
        assert not h.value
    # bad configs are rejected before touching any device
    assert lib.gsx_create(C.byref(abi.Config(n_topics=0, device=0)), C.byref(h)) == abi.GSX_EINVAL
    assert lib.gsx_create(C.byref(abi.Config(n_topics=65, device=0)), C.byref(h)) == abi.GSX_EINVAL


def test_null_engine_is_einval():
    lib = gsx.load_library()
    assert lib.gsx_refresh(None, 0) == abi.GSX_EINVAL
    assert lib.gsx_sync(None) == abi.GSX_EINVAL
    assert lib.gsx_destroy(None) == 0


@pytest.mark.parametrize("case", VAL["validation"], ids=[c["ref"] for c in VAL["validation"]])
def test_engine_params_validation(case):
    lib = gsx.load_library()
    if case["kind"] == "thresholds":
        ok = lib.gsx_validate_thresholds(C.byref(abi.Thresholds(**case["params"]))) == 0
    elif case["kind"] == "topic":
        ok = lib.gsx_validate_topic_params(C.byref(abi.TopicScoreParams(**case["params"]))) == 0
    else:
        ok = lib.gsx_validate_peer_params(C.byref(abi.PeerScoreParams(**case["params"]))) == 0
        ok = ok and all(lib.gsx_validate_topic_params(C.byref(abi.TopicScoreParams(**t))) == 0 for t in case["topics"])
    assert ok == case["valid"]


def test_engine_score_parameter_decay():
    lib = gsx.load_library()
    for c in VAL["decay"]:
        assert lib.gsx_score_parameter_decay(c["decay_ns"]) == c["expected"]
