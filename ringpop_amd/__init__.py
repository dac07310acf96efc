"""ringpop_amd — MI355X-native (gfx950 HIP) ringpop membership-convergence path.

The product is the C-ABI library libringpop_hip.so (include/ringpop_hip.h).
This package is the thin Python host binding used by the tests and bench.py;
the JavaScript drop-in surface lives in js/.  There is no CPU fallback: every
entry point runs on the GPU or raises.
"""
from ._lib import LIB_PATH, RingpopError, lib  # noqa: F401
from .farmhash import hash32, hash32_batch  # noqa: F401
from .hashring import HashRing  # noqa: F401
from .node import Dissemination, Membership, Node  # noqa: F401
from .sim import Sim  # noqa: F401

__all__ = ["Dissemination", "HashRing", "Membership", "Node", "RingpopError", "Sim", "hash32", "hash32_batch", "lib",
           "LIB_PATH"]
