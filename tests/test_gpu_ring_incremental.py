"""The drop-in ring's incremental updates (rp_capi.hip rp_ring::apply_delta,
rp_ring.hip k_ring_merge) against the C oracle's ring after every call.

The reference benchmarks addServer / removeServer one server at a time
(benchmarks/add-remove-hashring.js:35-52), and ringpop's update listener calls
addRemoveServers after every applied batch (lib/membership-update-listener.js);
a call touching at most RP_RING_INCR_MAX_POINTS replica points merges its
delta into the sorted point array instead of re-sorting every point.  Checked
here: the points (hash, owner name) and sampled lookups after every call, for
1,000 individual adds then removes with farmhash, for forced-collision hash
functions with mixed small batches (a server added and removed by one call,
removals of hashes another server owns, re-adds), and for an incremental call
right after a bulk build (the host mirror rebuilt from the device points).
lib/ring.js:39-94, lib/rbtree.js:70-232."""
import ctypes

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rp(gpu_lib):
    import ringpop_amd
    return ringpop_amd


def _blob(names):
    bs = [s.encode() for s in names]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs]) if bs else []
    blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
    return blob, off


class OracleRing:
    """The C oracle's ring (oracle/sim_oracle.c orc_ring_*), the checker."""

    def __init__(self, replicas, hash_func=None):
        self.L = oracle.lib()
        self.r = self.L.orc_ring_new(replicas)
        self.R = replicas
        self.hf = hash_func

    def _hashes(self, names):
        if self.hf is None or not names:
            return None
        return np.array([self.hf(f"{s}{i}") for s in names for i in range(self.R)], dtype=np.uint32)

    def add_remove(self, add, rm):
        ab, ao = _blob(add)
        rb, ro = _blob(rm)
        ah, rh = self._hashes(add), self._hashes(rm)
        return bool(self.L.orc_ring_add_remove(self.r, oracle._ptr(ab), oracle._ptr(ao), len(add),
                                               oracle._ptr(ah) if ah is not None else None, oracle._ptr(rb),
                                               oracle._ptr(ro), len(rm), oracle._ptr(rh) if rh is not None else None))

    def points(self):
        n = self.L.orc_ring_points(self.r, None, None)
        H = np.zeros(max(n, 1), dtype=np.uint32)
        O = np.zeros(max(n, 1), dtype=np.int32)
        self.L.orc_ring_points(self.r, oracle._ptr(H), oracle._ptr(O))
        buf = ctypes.create_string_buffer(512)
        names = {}
        for o in set(O[:n].tolist()):
            self.L.orc_ring_server_name(self.r, int(o), buf, 512)
            names[o] = buf.value.decode()
        return H[:n], [names[o] for o in O[:n].tolist()]

    def close(self):
        self.L.orc_ring_free(self.r)


def _same(ring, orc, probes):
    h, o = ring.points()
    oh, on = orc.points()
    assert np.array_equal(h, oh), (len(h), len(oh))
    assert [ring.server_name(int(x)) for x in o] == on
    if orc.hf is None:  # (with a hashFunc the checksum is hashFunc's, lib/ring.js:102)
        assert ring.checksum == oracle.lib().orc_ring_checksum(orc.r)
    if len(oh):  # lookups: the first point >= the probe, wrapping (lib/ring.js:138-147)
        idx = np.searchsorted(oh, probes, side="left")
        idx[idx == len(oh)] = 0
        got = ring.lookup_hashes(probes)
        assert [ring.server_name(int(x)) for x in got] == [on[i] for i in idx]


def _servers(n, port=3000):
    return [f"10.{i // 250}.{i % 250}.{1 + (i % 7)}:{port + i % 11}" for i in range(n)]


def test_individual_adds_then_removes_farmhash(rp):
    """benchmarks/add-remove-hashring.js's individual pattern: 1,000 addServer
    calls, then 1,000 removeServer calls in another order; the ring equals the
    oracle's after every call (every 50th: all points; every call: count,
    checksum and 64 probes)."""
    servers = _servers(1000)
    ring, orc = rp.HashRing(), OracleRing(100)
    rng = np.random.default_rng(11)
    probes = rng.integers(0, 2**32, size=64, dtype=np.uint64).astype(np.uint32)
    try:
        for i, s in enumerate(servers):
            ring.addServer(s)
            orc.add_remove([s], [])
            assert ring.getServerCount() == i + 1
            if i % 50 == 0 or i == len(servers) - 1:
                _same(ring, orc, probes)
            else:
                _, on = orc.points()
                got = ring.lookup_hashes(probes)
                oh, _ = orc.points()
                idx = np.searchsorted(oh, probes, side="left")
                idx[idx == len(oh)] = 0
                assert [ring.server_name(int(x)) for x in got] == [on[j] for j in idx]
        assert ring.checksum == oracle.lib().orc_ring_checksum(orc.r)
        for j, k in enumerate(rng.permutation(len(servers)).tolist()):
            ring.removeServer(servers[k])
            orc.add_remove([], [servers[k]])
            if j % 50 == 0 or j >= len(servers) - 3:
                _same(ring, orc, probes)
        h, _ = ring.points()
        assert len(h) == 0 and ring.getServerCount() == 0
        assert ring.lookup_hashes(probes).tolist() == [-1] * len(probes)
    finally:
        orc.close()
        ring.close()


@pytest.mark.parametrize("space", [3000, 400])
def test_forced_collisions_mixed_batches(rp, space):
    """A hashFunc folding replica names into `space` values (lib/ring.js:29):
    most replica hashes collide, so inserts keep the first inserter, removals
    erase points other servers own, and re-added servers find their hashes
    taken.  Random small addRemoveServers calls (1-4 adds, 0-3 removes, a
    server sometimes added and removed by the same call) against the oracle
    after every call."""
    import zlib

    def hf(s):
        return (zlib.crc32(s.encode()) % space) * 7919 + 13

    servers = _servers(120, port=4000)
    ring, orc = rp.HashRing(replica_points=20, hash_func=hf), OracleRing(20, hash_func=hf)
    rng = np.random.default_rng(space)
    probes = rng.integers(0, space * 7919 + 14, size=48).astype(np.uint32)
    present = set()
    try:
        for step in range(300):
            add = [servers[i] for i in rng.choice(len(servers), size=int(rng.integers(1, 5)), replace=False)]
            pool = sorted(present | set(add))
            k = int(rng.integers(0, 4))
            rm = [pool[i] for i in rng.choice(len(pool), size=min(k, len(pool)), replace=False)] if pool else []
            if step % 7 == 3:
                rm = rm + [add[0]]  # added and removed by one call
            assert ring.addRemoveServers(add, rm) == orc.add_remove(add, rm), step
            present = (present | set(add)) - set(rm)
            assert ring.getServerCount() == len(present)
            _same(ring, orc, probes)
    finally:
        orc.close()
        ring.close()


def test_incremental_after_bulk_build(rp):
    """A bulk build (10,000 servers: device replica hashing and radix sort),
    then single-server adds and removes (the incremental path rebuilds its
    host mirror from the device points first), against the oracle."""
    servers = _servers(10_050)
    ring, orc = rp.HashRing(), OracleRing(100)
    rng = np.random.default_rng(5)
    probes = rng.integers(0, 2**32, size=256, dtype=np.uint64).astype(np.uint32)
    try:
        ring.addRemoveServers(servers[:10_000], None)
        orc.add_remove(servers[:10_000], [])
        _same(ring, orc, probes)
        for s in servers[10_000:10_020]:
            ring.addServer(s)
            orc.add_remove([s], [])
        _same(ring, orc, probes)
        for s in servers[:10]:
            ring.removeServer(s)
            orc.add_remove([], [s])
        ring.addRemoveServers(servers[10_020:10_050], servers[10:40])
        orc.add_remove(servers[10_020:10_050], servers[10:40])
        _same(ring, orc, probes)
        assert ring.checksum == oracle.lib().orc_ring_checksum(orc.r)
    finally:
        orc.close()
        ring.close()


def test_update_waits_for_queued_device_lookups(rp):
    """a device lookup queued on a caller's stream (rp_stream_create:
    non-blocking) and not yet synchronised, then addServer / removeServer on
    the incremental path, which rewrites the points and lookup directories in
    place on the null stream.  The update must wait for the lookup: every
    queued lookup answers the ring as it was, and a lookup after the update
    answers the new ring (against the oracle)."""
    import ctypes

    from ringpop_amd import hiprt
    from ringpop_amd._lib import check, lib
    L = lib()
    servers = _servers(10_004)
    ring, orc = rp.HashRing(), OracleRing(100)
    try:
        ring.addRemoveServers(servers[:10_000], None)
        orc.add_remove(servers[:10_000], [])
        n, seed = 50_000_000, 7
        d_bytes, d_off, total = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        check(L.rp_ring_make_keys_device(ring._h, seed, n, ctypes.byref(d_bytes), ctypes.byref(d_off),
                                         ctypes.byref(total)))
        before = hiprt.DeviceArray(n, np.int32)
        check(L.rp_ring_lookup_batch_device(ring._h, d_bytes, d_off, n, before.ptr, None))
        want_before = before.numpy()
        st = hiprt.Stream()
        outs = [hiprt.DeviceArray(n, np.int32) for _ in range(2)]
        for o in outs:  # queued, not synchronised
            check(L.rp_ring_lookup_batch_device(ring._h, d_bytes, d_off, n, o.ptr, st.handle))
        ring.addServer(servers[10_000])
        ring.removeServer(servers[0])
        orc.add_remove([servers[10_000]], [])
        orc.add_remove([], [servers[0]])
        after = hiprt.DeviceArray(n, np.int32)
        check(L.rp_ring_lookup_batch_device(ring._h, d_bytes, d_off, n, after.ptr, st.handle))
        st.synchronize()
        for o in outs:
            assert np.array_equal(o.numpy(), want_before)
        got_after = after.numpy()
        idx = np.random.default_rng(3).integers(0, n, size=100_000)
        keys = oracle.lookup_keys(seed, idx)
        ph, pnames = orc.points()
        ix = np.searchsorted(ph, oracle.farmhash32_batch(keys), side="left")
        ix[ix == len(ph)] = 0
        names = {int(x): ring.server_name(int(x)) for x in np.unique(got_after[idx])}
        assert [names[int(x)] for x in got_after[idx]] == [pnames[i] for i in ix]
        assert (got_after != want_before).any()  # (the ring did change)
        for b in outs + [before, after]:
            b.free()
        st.destroy()
    finally:
        orc.close()
        ring.close()


@pytest.mark.parametrize("extra", [-40, -1, 0, 1, 15, 16, 17, 600])
def test_checksum_around_host_stage_limit(rp, extra):
    """The ring checksum (lib/ring.js:96-105) of server strings around
    HASH_HOST_MAX = 48 KB, where rp_ring_checksum switches from k_hash_host
    (the string read over PCIe into LDS) to a staging copy and k_hash_one:
    1,480 names of 32 bytes and one whose length puts the ';'-joined string at
    48 KB + extra, against the oracle."""
    limit = 48 * 1024
    names = [f"10.9.{i // 250}.{i % 250}:{30000 + i:05d}-pad-pad-pad"[:32].ljust(32, "x") for i in range(1480)]
    k = limit + extra - (32 * 1480 + 1480)
    assert k > 0
    names.append("z" * k)
    assert len(";".join(sorted(names))) == limit + extra
    ring, orc = rp.HashRing(replica_points=1), OracleRing(1)
    try:
        ring.addRemoveServers(names, None)
        orc.add_remove(names, [])
        assert ring.checksum == oracle.lib().orc_ring_checksum(orc.r)
        ring.removeServer(names[7])  # (33 bytes shorter, through the incremental path)
        orc.add_remove([], [names[7]])
        assert ring.checksum == oracle.lib().orc_ring_checksum(orc.r)
    finally:
        orc.close()
        ring.close()
