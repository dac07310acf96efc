import gzip
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libringpop_hip.so)")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    p = os.path.join(GOLDEN, name)
    if name.endswith(".gz"):
        with gzip.open(p, "rt") as f:
            return json.load(f)
    with open(p) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real GPU; builds it if needed."""
    import ringpop_amd
    from ringpop_amd import build
    build.build()
    lib = ringpop_amd.lib()
    return lib
