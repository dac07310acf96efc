"""farmhash.hash32 on the GPU (replaces npm `farmhash` ^0.2.0, package.json:30).

`hash32(string)` mirrors the npm module's single entry point used by the
reference (lib/membership.js:57, lib/ring.js:29); `hash32_batch` is the
batched form the device path is built for.
"""
import ctypes

import numpy as np

from ._lib import check, lib, ptr


def _encode(strings):
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    blob = np.frombuffer(b"".join(bs) + b"\0" * 8, dtype=np.uint8)
    return blob, off


def hash32(s):
    b = s.encode() if isinstance(s, str) else bytes(s)
    out = ctypes.c_uint32(0)
    buf = ctypes.create_string_buffer(b, len(b) + 1)
    check(lib().rp_hash32(ctypes.cast(buf, ctypes.c_void_p), len(b), ctypes.byref(out)))
    return out.value


def hash32_batch(strings):
    blob, off = _encode(strings)
    out = np.zeros(len(off) - 1, dtype=np.uint32)
    if len(out):
        check(lib().rp_hash32_batch(ptr(blob), ptr(off), len(out), ptr(out)))
    return out
