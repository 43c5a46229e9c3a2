import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "go-libp2p-pubsub_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs through the C ABI of libgsx.so")
    config.addinivalue_line("markers", "slow: long-running")


def _make(d):
    subprocess.run(["make", "-s", "-C", d], check=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    """The oracle (checker) and the engine library are built in-tree; make is incremental."""
    _make(os.path.join(ROOT, "oracle"))
    _make(PKG)
    yield


@pytest.fixture(scope="session")
def gpu_ok():
    import gsx

    lib = gsx.load_library()
    import ctypes as C

    cfg = gsx.abi.Config(n_topics=1, device=0)
    h = C.c_void_p()
    rc = lib.gsx_create(C.byref(cfg), C.byref(h))
    if rc != 0:
        pytest.fail(f"gsx_create failed with {rc}: a gpu-marked test needs a gfx950 device")
    lib.gsx_destroy(h)
    return True
