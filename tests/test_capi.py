"""CPU tests of the boundary: the C-ABI library builds, loads and exports every
symbol include/ringpop_hip.h declares (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ringpop_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rp_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("rp_hash32", "rp_hash32_batch", "rp_ring_create", "rp_ring_lookup_batch", "rp_sim_create",
              "rp_sim_round", "rp_sim_read_checksums", "rp_sim_destroy"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from ringpop_amd import build
    path = build.build()
    L = ctypes.CDLL(path)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from ringpop_amd import _lib
    assert set(declared_symbols()) == set(_lib.SIGNATURES)


def test_no_gpu_fails_loudly():
    """Without a GPU the product raises instead of falling back to the CPU."""
    import ringpop_amd
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(ringpop_amd.RingpopError):
        ringpop_amd.hash32("abc")
    with pytest.raises(ringpop_amd.RingpopError):
        ringpop_amd.Sim(16, 1)
