"""Device buffers, streams and events through libringpop_hip.so's own HIP
runtime (rp_device_* / rp_stream_* / rp_event_*), for callers of the batched
*_device entry points (bench.py, tests).  Plumbing only: going through the
library guarantees the same runtime as its kernels, whatever else (torch's
bundled runtime, say) the process has loaded.
"""
import ctypes

import numpy as np

from ._lib import check, lib

H2D, D2H, D2D = 1, 2, 3


class DeviceArray:
    """A device allocation of `n` elements of numpy `dtype`."""

    def __init__(self, n, dtype):
        self.n, self.dtype = int(n), np.dtype(dtype)
        self.ptr = ctypes.c_void_p()
        check(lib().rp_device_malloc(max(self.n, 1) * self.dtype.itemsize, ctypes.byref(self.ptr)))

    @property
    def nbytes(self):
        return self.n * self.dtype.itemsize

    def numpy(self):
        out = np.empty(self.n, dtype=self.dtype)
        check(lib().rp_device_synchronize())
        check(lib().rp_device_memcpy(ctypes.c_void_p(out.ctypes.data), self.ptr, self.nbytes, D2H))
        return out

    def free(self):
        if self.ptr:
            lib().rp_device_free(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def synchronize():
    check(lib().rp_device_synchronize())


class Stream:
    def __init__(self):
        self.handle = ctypes.c_void_p()
        check(lib().rp_stream_create(ctypes.byref(self.handle)))

    def synchronize(self):
        check(lib().rp_stream_synchronize(self.handle))

    def destroy(self):
        if self.handle:
            lib().rp_stream_destroy(self.handle)
            self.handle = ctypes.c_void_p()


class Event:
    def __init__(self):
        self.handle = ctypes.c_void_p()
        check(lib().rp_event_create(ctypes.byref(self.handle)))

    def record(self, stream):
        check(lib().rp_event_record(self.handle, stream.handle))

    def elapsed_ms(self, end):
        ms = ctypes.c_float(0)
        check(lib().rp_event_elapsed_ms(self.handle, end.handle, ctypes.byref(ms)))
        return ms.value

    def destroy(self):
        if self.handle:
            lib().rp_event_destroy(self.handle)
            self.handle = ctypes.c_void_p()


def memory():
    """(free, total) bytes of the current device (rp_device_memory)."""
    f, t = ctypes.c_size_t(0), ctypes.c_size_t(0)
    check(lib().rp_device_memory(ctypes.byref(f), ctypes.byref(t)))
    return f.value, t.value
