"""HashRing with the reference's API (lib/ring.js:25-184), points kept on the GPU.

Method names and semantics follow lib/ring.js: addServer / removeServer /
addRemoveServers (adds first, then removes; returns whether the ring
changed), hasServer, getServerCount, computeChecksum (checksum attribute),
lookup (inclusive lower bound with wrap, None on an empty ring) and lookupN.
`hash_func` mirrors the `hashFunc` option (lib/ring.js:29): when given, replica
and key hashes are computed by it on the host and only the ring runs on the
device.  Batched `lookup_batch` is the device-native entry point.
"""
import ctypes

import numpy as np

from ._lib import check, lib, ptr
from .farmhash import _encode


class HashRing:
    def __init__(self, replica_points=100, hash_func=None):
        self.replica_points = replica_points or 100
        self.hash_func = hash_func
        self._h = ctypes.c_void_p()
        check(lib().rp_ring_create(self.replica_points, ctypes.byref(self._h)))
        self.checksum = None
        self.servers = {}

    def close(self):
        if self._h:
            lib().rp_ring_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _hashes(self, names):
        if self.hash_func is None or not names:
            return None
        return np.array([self.hash_func(f"{s}{i}") for s in names for i in range(self.replica_points)],
                        dtype=np.uint32)

    def addRemoveServers(self, servers_to_add=None, servers_to_remove=None):
        add = list(servers_to_add or [])
        rm = list(servers_to_remove or [])
        ab, ao = _encode(add)
        rb, ro = _encode(rm)
        ah, rh = self._hashes(add), self._hashes(rm)
        changed = ctypes.c_int(0)
        check(lib().rp_ring_add_remove(self._h, ptr(ab), ptr(ao), len(add), ptr(ah), ptr(rb), ptr(ro), len(rm),
                                       ptr(rh), ctypes.byref(changed)))
        for s in add:
            self.servers[s] = True
        for s in rm:
            self.servers.pop(s, None)
        if changed.value:
            self.computeChecksum()
        return bool(changed.value)

    def addServer(self, name):
        if self.hasServer(name):
            return
        self.addRemoveServers([name], None)

    def removeServer(self, name):
        if not self.hasServer(name):
            return
        self.addRemoveServers(None, [name])

    def hasServer(self, name):
        b = name.encode()
        out = ctypes.c_int(0)
        check(lib().rp_ring_has_server(self._h, ctypes.c_char_p(b), len(b), ctypes.byref(out)))
        return bool(out.value)

    def getServerCount(self):
        out = ctypes.c_int(0)
        check(lib().rp_ring_server_count(self._h, ctypes.byref(out)))
        return out.value

    def computeChecksum(self):
        out = ctypes.c_uint32(0)
        if self.hash_func is not None:
            self.checksum = self.hash_func(";".join(sorted(self.servers)))
            return self.checksum
        check(lib().rp_ring_checksum(self._h, ctypes.byref(out)))
        self.checksum = out.value
        return self.checksum

    def server_name(self, idx):
        if idx < 0:
            return None
        buf = ctypes.create_string_buffer(512)
        n = ctypes.c_size_t(0)
        check(lib().rp_ring_server_name(self._h, int(idx), buf, 512, ctypes.byref(n)))
        return buf.value.decode()

    def lookup_batch(self, keys):
        """Owner server index per key (device farmhash + lower bound); -1 on an empty ring."""
        keys = list(keys)
        if self.hash_func is not None:
            return self.lookup_hashes(np.array([self.hash_func(k) for k in keys], dtype=np.uint32))
        blob, off = _encode(keys)
        out = np.zeros(len(keys), dtype=np.int32)
        if keys:
            check(lib().rp_ring_lookup_batch(self._h, ptr(blob), ptr(off), len(keys), ptr(out)))
        return out

    lookup_indices = lookup_batch

    def lookup_hashes(self, hashes):
        h = np.ascontiguousarray(hashes, dtype=np.uint32)
        out = np.zeros(len(h), dtype=np.int32)
        if len(h):
            check(lib().rp_ring_lookup_hashes(self._h, ptr(h), len(h), ptr(out)))
        return out

    def lookup(self, key):
        return self.server_name(int(self.lookup_batch([str(key)])[0]))

    def lookupN(self, key, n):
        if self.hash_func is not None:
            h = np.array([self.hash_func(str(key))], dtype=np.uint32)
        else:
            from .farmhash import hash32_batch
            h = hash32_batch([str(key)])
        out = np.full(max(n, 1), -1, dtype=np.int32)
        cnt = np.zeros(1, dtype=np.int32)
        check(lib().rp_ring_lookup_n_hashes(self._h, ptr(h), 1, int(n), ptr(out), ptr(cnt)))
        return [self.server_name(int(x)) for x in out[: int(cnt[0])]]

    def group_indices(self, keys):
        """Device grouping of `keys` by owner: (dests, group_off, key_index) arrays.

        handleOrProxyAll (index.js:636-645) groups with ``_.groupBy(keys,
        this.lookup)``: groups in first-appearance order of their owner, keys
        in input order; dests[g] is a server index (-1 on an empty ring).
        """
        keys = list(keys)
        n = len(keys)
        dests = np.zeros(max(n, 1), dtype=np.int32)
        goff = np.zeros(n + 1, dtype=np.uint32)
        kidx = np.zeros(max(n, 1), dtype=np.uint32)
        ng = ctypes.c_size_t(0)
        if self.hash_func is not None:
            h = np.array([self.hash_func(str(k)) for k in keys], dtype=np.uint32)
            check(lib().rp_ring_group_hashes(self._h, ptr(h), n, ptr(dests), ptr(goff), ptr(kidx),
                                             ctypes.byref(ng)))
        else:
            blob, off = _encode([str(k) for k in keys])
            check(lib().rp_ring_group_keys(self._h, ptr(blob), ptr(off), n, ptr(dests), ptr(goff), ptr(kidx),
                                           ctypes.byref(ng)))
        g = ng.value
        return dests[:g], goff[: g + 1], kidx[:n]

    def groupByOwner(self, keys):
        """``_.groupBy(keys, ring.lookup)`` as handleOrProxyAll builds it: an
        insertion-ordered dict {dest address (None on an empty ring): [keys]}."""
        keys = list(keys)
        dests, goff, kidx = self.group_indices(keys)
        return {self.server_name(int(d)): [keys[int(i)] for i in kidx[goff[g]:goff[g + 1]]]
                for g, d in enumerate(dests)}

    def points(self):
        n = ctypes.c_size_t(0)
        check(lib().rp_ring_points(self._h, None, None, 0, ctypes.byref(n)))
        h = np.zeros(n.value, dtype=np.uint32)
        o = np.zeros(n.value, dtype=np.int32)
        if n.value:
            check(lib().rp_ring_points(self._h, ptr(h), ptr(o), n.value, ctypes.byref(n)))
        return h, o
