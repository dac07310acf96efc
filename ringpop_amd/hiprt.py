"""Minimal ctypes access to the HIP runtime libringpop_hip.so itself uses.

Device buffers, streams and events for the batched *_device entry points
(bench.py, tests).  This is plumbing: it loads /opt/rocm's libamdhip64 -- the
runtime the product library links -- so a buffer allocated here is valid for
the library's kernels in the same process.
"""
import ctypes
import os

import numpy as np

_hip = None
H2D, D2H, D2D = 1, 2, 3


def hip():
    global _hip
    if _hip is None:
        path = "/opt/rocm/lib/libamdhip64.so"
        _hip = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        _hip.hipGetErrorString.restype = ctypes.c_char_p
    return _hip


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {hip().hipGetErrorString(rc).decode()}")


class DeviceArray:
    """A device allocation of `n` elements of numpy `dtype`."""

    def __init__(self, n, dtype):
        self.n, self.dtype = int(n), np.dtype(dtype)
        self.ptr = ctypes.c_void_p()
        _ok(hip().hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(max(self.n, 1) * self.dtype.itemsize)), "hipMalloc")

    @property
    def nbytes(self):
        return self.n * self.dtype.itemsize

    def numpy(self):
        out = np.empty(self.n, dtype=self.dtype)
        synchronize()
        _ok(hip().hipMemcpy(ctypes.c_void_p(out.ctypes.data), self.ptr, ctypes.c_size_t(self.nbytes), D2H), "hipMemcpy")
        return out

    def free(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def synchronize():
    _ok(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")


class Stream:
    def __init__(self):
        self.handle = ctypes.c_void_p()
        _ok(hip().hipStreamCreate(ctypes.byref(self.handle)), "hipStreamCreate")

    def synchronize(self):
        _ok(hip().hipStreamSynchronize(self.handle), "hipStreamSynchronize")

    def destroy(self):
        if self.handle:
            hip().hipStreamDestroy(self.handle)
            self.handle = ctypes.c_void_p()


class Event:
    def __init__(self):
        self.handle = ctypes.c_void_p()
        _ok(hip().hipEventCreate(ctypes.byref(self.handle)), "hipEventCreate")

    def record(self, stream):
        _ok(hip().hipEventRecord(self.handle, stream.handle), "hipEventRecord")

    def elapsed_ms(self, end):
        ms = ctypes.c_float(0)
        _ok(hip().hipEventElapsedTime(ctypes.byref(ms), self.handle, end.handle), "hipEventElapsedTime")
        return ms.value

    def destroy(self):
        if self.handle:
            hip().hipEventDestroy(self.handle)
            self.handle = ctypes.c_void_p()
