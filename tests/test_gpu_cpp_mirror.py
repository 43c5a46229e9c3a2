"""The reference's score_test.go restated in C++ over include/gsx_pubsub.hpp
(the host-side mirror of the peerScore interface), run on the GPU engine."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "score_test.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "score_test")
LIBDIR = os.path.join(ROOT, "go-libp2p-pubsub_amd", "gsx")


def build():
    subprocess.run(
        ["g++", "-std=c++17", "-O1", "-Wall", "-ffp-contract=off", SRC, f"-L{LIBDIR}", "-lgsx",
         f"-Wl,-rpath,{LIBDIR}", "-o", BIN],
        check=True,
    )


def test_cpp_mirror_compiles():
    build()
    assert os.path.exists(BIN)


@pytest.mark.gpu
def test_cpp_mirror_score_tests(gpu_ok):
    build()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout
