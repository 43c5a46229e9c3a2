"""gsx — MI355X-native GossipSub scoring engine (Python handle on libgsx.so).

The engine is the HIP library built from ../csrc; this package only loads it
(abi), drives it (engine) and builds seeded synthetic inputs (synth).
"""
from . import abi  # noqa: F401
from .abi import GsxError, load_library  # noqa: F401
from .engine import Engine, make_struct  # noqa: F401
