"""TEST INFRASTRUCTURE ONLY: ctypes loader for the CPU oracle (oracle/build/liboracle.so).

The oracle is the C restatement of the reference's hot path (see
oracle/sim_oracle.c for reference file:line citations).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker -- the product (ringpop_amd) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c = ctypes
        P = c.c_void_p
        L.oracle_farmhash32.restype = c.c_uint32
        L.oracle_farmhash32.argtypes = [c.c_char_p, c.c_size_t]
        L.oracle_farmhash32_seed.restype = c.c_uint32
        L.oracle_farmhash32_seed.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32]
        L.oracle_farmhash_test_seed.restype = c.c_uint32
        L.oracle_farmhash_test_seed.argtypes = [c.c_int, c.c_int]
        L.oracle_farmhash32_batch.argtypes = [P, P, c.c_size_t, P]
        L.orc_sim_new.restype = P
        L.orc_sim_new.argtypes = [c.c_int, c.c_uint64, c.c_int, c.c_int]
        L.orc_sim_new2.restype = P
        L.orc_sim_new2.argtypes = [c.c_int, c.c_uint64, c.c_int, c.c_int, c.c_int]
        L.orc_sim_new3.restype = P
        L.orc_sim_new3.argtypes = [c.c_int, c.c_uint64, c.c_int, c.c_int, c.c_int, P, P, P, P]
        L.orc_sim_join.restype = c.c_int
        L.orc_sim_join.argtypes = [P, P, P, P, c.c_int, c.c_int]
        L.orc_sim_free.argtypes = [P]
        L.orc_sim_fail.argtypes = [P, c.c_int, c.c_int]
        L.orc_sim_partition.argtypes = [P, c.c_int, c.c_int, c.c_int]
        L.orc_sim_storm.argtypes = [P, c.c_int, c.c_int, c.c_int]
        L.orc_sim_round.argtypes = [P, c.c_int, P, P, P]
        L.orc_sim_checksum.restype = c.c_uint32
        L.orc_sim_checksum.argtypes = [P, c.c_int]
        L.orc_sim_is_dead.argtypes = [P, c.c_int]
        L.orc_sim_dump_view.argtypes = [P, c.c_int, P, P]
        L.orc_sim_dump_members.argtypes = [P, c.c_int, P]
        L.orc_sim_dump_changes.argtypes = [P, c.c_int, P]
        L.orc_sim_node_info.argtypes = [P, c.c_int, P]
        L.orc_sim_dump_timers.argtypes = [P, c.c_int, P]
        L.orc_sim_ring_lookup.argtypes = [P, c.c_int, c.c_uint32]
        L.orc_sim_address.argtypes = [P, c.c_int, c.c_char_p, c.c_int]
        L.orc_ring_new.restype = P
        L.orc_ring_new.argtypes = [c.c_int]
        L.orc_ring_free.argtypes = [P]
        L.orc_ring_add_remove.argtypes = [P, P, P, c.c_int, P, P, P, c.c_int, P]
        L.orc_ring_server_count.argtypes = [P]
        L.orc_ring_checksum.restype = c.c_uint32
        L.orc_ring_checksum.argtypes = [P]
        L.orc_ring_lookup_hashes.argtypes = [P, P, c.c_size_t, P]
        L.orc_ring_points.restype = c.c_size_t
        L.orc_ring_points.argtypes = [P, P, P]
        L.orc_ring_server_name.argtypes = [P, c.c_int, c.c_char_p, c.c_int]
        L.orc_ring_lookup_n.argtypes = [P, c.c_uint32, c.c_int, P]
        L.orc_view_update.argtypes = [c.c_int, c.c_uint64, P, P, c.c_int, P, P, P, P]
        L.orc_checksum_string.restype = c.c_size_t
        L.orc_checksum_string.argtypes = [P, P, c.c_int, P, P, P, c.c_size_t]
        L.orc_view_checksum.restype = c.c_uint32
        L.orc_view_checksum.argtypes = [P, P, c.c_int, P, P]
        L.orc_max_piggyback.argtypes = [c.c_int, c.c_int]
        L.orc_sim_ping_body.argtypes = [P, c.c_int, P, c.c_int, P, P]
        L.orc_sim_handle_ping.argtypes = [P, c.c_int, c.c_int, c.c_uint64, c.c_uint32, P, c.c_int, P, c.c_int, P, P]
        L.orc_sim_update.argtypes = [P, c.c_int, P, c.c_int]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def farmhash32(data):
    if isinstance(data, str):
        data = data.encode()
    return lib().oracle_farmhash32(data, len(data))


def farmhash32_batch(strings):
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
    out = np.zeros(len(bs), dtype=np.uint32)
    lib().oracle_farmhash32_batch(_ptr(blob), _ptr(off), len(bs), _ptr(out))
    return out


class Stats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in
                ("evaluated", "applied", "full_syncs", "messages", "waves", "converged")]


class Sim:
    """The oracle simulation: N reference-semantics nodes, CPU, sequential."""

    def __init__(self, n, seed, churn_k=None, eager=False, failures=None, partition=None, replica_hash_shift=0,
                 storm=None, addresses=None, views=None, joins=None):
        """addresses: n address strings in sort order; views: (status, inc)
        (n, n) arrays of the bootstrap's views (orc_sim_new3); joins:
        [(round, joiner, [seeds])] (orc_sim_join; the others start with
        views of each other)."""
        self.n = n
        self.churn_k = churn_k if churn_k is not None else -(-n // 100)
        if joins and views is None:
            member = np.ones(n, dtype=np.uint8)
            member[[j[1] for j in joins]] = 0
            views = (np.tile(member, (n, 1)), np.tile(1434401518824 + np.arange(n, dtype=np.uint64), (n, 1)))
            views[0][np.arange(n), np.arange(n)] = 1
        if addresses is None and views is None:
            self.h = lib().orc_sim_new2(n, seed, self.churn_k, 1 if eager else 0, replica_hash_shift)
        else:
            ab = ao = vs = vi = None
            if addresses is not None:
                bs = [a.encode() for a in addresses]
                ao = np.zeros(n + 1, dtype=np.uint64)
                ao[1:] = np.cumsum([len(b) for b in bs])
                ab = np.frombuffer(b"".join(bs), dtype=np.uint8)
            if views is not None:
                vs = np.ascontiguousarray(views[0], dtype=np.uint8)
                vi = np.ascontiguousarray(views[1], dtype=np.uint64)
            self._keep = (ab, ao, vs, vi)
            self.h = lib().orc_sim_new3(n, seed, self.churn_k, 1 if eager else 0, replica_hash_shift,
                                        _ptr(ab), _ptr(ao), _ptr(vs), _ptr(vi))
        if joins:
            sp = max([len(j[2]) for j in joins] + [1])
            ids = np.array([j[1] for j in joins], dtype=np.int32)
            rounds = np.array([j[0] for j in joins], dtype=np.int32)
            seeds = np.full((len(joins), sp), -1, dtype=np.int32)
            for i, j in enumerate(joins):
                seeds[i, :len(j[2])] = j[2]
            assert lib().orc_sim_join(self.h, _ptr(ids), _ptr(rounds), _ptr(seeds), len(joins), sp) == 0
        for rnd, ids in (failures or {}).items():
            for v in ids:
                lib().orc_sim_fail(self.h, int(v), int(rnd))
        if partition:
            lib().orc_sim_partition(self.h, partition["start"], partition["end"], partition["split"])
        if storm:
            lib().orc_sim_storm(self.h, storm["start"], storm["end"], storm["ppm"])

    def close(self):
        if self.h:
            lib().orc_sim_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def round(self, churn=True):
        st = Stats()
        ch = np.zeros(max(self.churn_k, 1), dtype=np.int32)
        nc = ctypes.c_int(0)
        lib().orc_sim_round(self.h, 1 if churn else 0, ctypes.byref(st), _ptr(ch), ctypes.byref(nc))
        d = {k: getattr(st, k) for k, _ in Stats._fields_}
        d["churned"] = ch[: nc.value].tolist()
        return d

    def checksum(self, v):
        return lib().orc_sim_checksum(self.h, v)

    def checksums(self):
        return [None if lib().orc_sim_is_dead(self.h, v) else self.checksum(v) for v in range(self.n)]

    def view(self, v):
        st = np.zeros(self.n, dtype=np.uint8)
        inc = np.zeros(self.n, dtype=np.uint64)
        lib().orc_sim_dump_view(self.h, v, _ptr(st), _ptr(inc))
        return st, inc

    def members(self, v):
        out = np.zeros(self.n, dtype=np.int32)
        k = lib().orc_sim_dump_members(self.h, v, _ptr(out))
        return out[:k]

    def changes(self, v):
        out = np.zeros((self.n, 6), dtype=np.int64)
        k = lib().orc_sim_dump_changes(self.h, v, _ptr(out))
        return out[:k]

    def info(self, v):
        out = np.zeros(8, dtype=np.int64)
        lib().orc_sim_node_info(self.h, v, _ptr(out))
        keys = ("max_pb", "ring_servers", "ring_checksum", "iter_index", "iter_round", "dead", "rng", "timers")
        return dict(zip(keys, out.tolist()))

    def timers(self, v):
        out = np.zeros(self.n, dtype=np.int32)
        k = lib().orc_sim_dump_timers(self.h, v, _ptr(out))
        return out[:k]

    def ring_lookup(self, v, h):
        return lib().orc_sim_ring_lookup(self.h, v, h)

    def address(self, i):
        b = ctypes.create_string_buffer(64)
        lib().orc_sim_address(self.h, i, b, 64)
        return b.value.decode()

    # wire bridge (rows: address, status, incarnation, source, source inc)
    def ping_body(self, v):
        out = np.zeros((self.n, 5), dtype=np.int64)
        cs, inc = ctypes.c_uint32(0), ctypes.c_uint64(0)
        k = lib().orc_sim_ping_body(self.h, v, _ptr(out), self.n, ctypes.byref(cs), ctypes.byref(inc))
        return out[:k], cs.value, inc.value

    def handle_ping(self, v, source, source_inc, checksum, rows):
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64).reshape(-1, 5))
        out = np.zeros((self.n, 5), dtype=np.int64)
        ap, fs = ctypes.c_int(0), ctypes.c_int(0)
        k = lib().orc_sim_handle_ping(self.h, v, int(source), int(source_inc), int(checksum) & 0xFFFFFFFF, _ptr(r),
                                      len(r), _ptr(out), self.n, ctypes.byref(ap), ctypes.byref(fs))
        return out[:k], ap.value, bool(fs.value)

    def update(self, v, rows):
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64).reshape(-1, 5))
        return lib().orc_sim_update(self.h, v, _ptr(r), len(r))


def max_piggyback(server_count, factor=15):
    return lib().orc_max_piggyback(server_count, factor)


def ring_points_add_only(names, replica_points=100):
    """Sorted (hash, owner index) points of a HashRing built by one
    addRemoveServers(names, []) call (lib/ring.js:60-75): replica i of server s
    hashes farmhash32(s + i) (lib/ring.js:128-131) and RBTree.insert keeps the
    first inserter of a duplicate hash (lib/rbtree.js:112-117).  numpy
    restatement for large rings (the C oracle's array insert is O(P^2))."""
    reps = [f"{s}{i}" for s in names for i in range(replica_points)]
    h = farmhash32_batch(reps)
    owner = np.repeat(np.arange(len(names), dtype=np.int32), replica_points)
    order = np.argsort(h, kind="stable")  # insertion order kept among equal hashes
    hs, os_ = h[order], owner[order]
    first = np.ones(len(hs), dtype=bool)
    first[1:] = hs[1:] != hs[:-1]
    return hs[first], os_[first]


def ring_lookup_points(points_h, points_owner, key_hashes):
    """HashRing.lookup (lib/ring.js:138-147): first point with hash >= key
    (RBTree.lowerBound, lib/rbtree.js:235-260), else the minimum point."""
    if len(points_h) == 0:
        return np.full(len(key_hashes), -1, dtype=np.int32)
    p = np.searchsorted(points_h, np.asarray(key_hashes, dtype=np.uint32), side="left")
    p[p == len(points_h)] = 0
    return points_owner[p]


def lookup_keys(seed, idx):
    """Config-3 synthetic keys (decimal strings of splitmix64 values), the same
    definition as the device generator rp_ring_make_keys_device."""
    G = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        s = np.uint64(seed) + np.asarray(idx, dtype=np.uint64) * G + G
        z = (s ^ (s >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return [str(int(x)) for x in z]


def group_by_owner(owners):
    """handleOrProxyAll's ``_.groupBy(keys, this.lookup)`` then
    ``Object.keys(keysByDest)`` (index.js:642-643): groups in first-appearance
    order of their owner (string object keys keep insertion order), key
    indices within a group in input order.  underscore's groupBy (not
    vendored in the reference) pushes each element onto result[key] in one
    pass over the list; an empty ring's null owner is the key "null" (-1
    here).  Returns (dests, group_off, key_index) like rp_ring_group_*."""
    groups = {}
    for i, o in enumerate(np.asarray(owners, dtype=np.int64).tolist()):
        groups.setdefault(o, []).append(i)
    dests = np.array(list(groups), dtype=np.int32)
    lens = [len(v) for v in groups.values()]
    goff = np.zeros(len(lens) + 1, dtype=np.uint32)
    goff[1:] = np.cumsum(lens, dtype=np.uint64)
    kidx = np.array([i for v in groups.values() for i in v], dtype=np.uint32)
    return dests, goff, kidx


def group_by_owner_np(owners):
    """group_by_owner for large batches (stable argsort; same result)."""
    o = np.asarray(owners, dtype=np.int64)
    if len(o) == 0:
        return np.zeros(0, np.int32), np.zeros(1, np.uint32), np.zeros(0, np.uint32)
    order = np.argsort(o, kind="stable")
    so = o[order]
    head = np.ones(len(so), dtype=bool)
    head[1:] = so[1:] != so[:-1]
    starts = np.flatnonzero(head)
    ends = np.append(starts[1:], len(so))
    first = order[starts]  # first key index of each owner
    g = np.argsort(first, kind="stable")
    dests = so[starts][g].astype(np.int32)
    lens = (ends - starts)[g]
    goff = np.zeros(len(g) + 1, dtype=np.uint32)
    goff[1:] = np.cumsum(lens)
    kidx = np.concatenate([order[starts[r]:ends[r]] for r in g]).astype(np.uint32)
    return dests, goff, kidx
