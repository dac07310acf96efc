"""GPU correctness at the benchmarked sizes (configs 3, 4 and 5).

The headline runs at N = 65,536: 2^32 view cells, so index-width, arena,
seen-window and origin-table sizing bugs that small runs cannot reach would
show here.  Checks that do not need a CPU run of the same size:
  * sampled checksums recomputed on the host from the device's views with the
    oracle's checksum string + farmhash (lib/membership.js:41-93),
  * dissemination-table invariants (lib/dissemination.js: distinct keys,
    piggyback counts <= maxPiggybackCount, every recorded change equals the
    member it was applied to, valid sources),
  * 1 shard == 4 in-process shards, round by round,
  * config 5's end state (every fail-stopped node faulty in every live view,
    every false suspicion refuted, every live ring holds the live servers),
and at N = 8,192 the oracle itself through a committed fixture
(oracle/gen_large_fixture.py).
"""
import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

N = 65536


@pytest.fixture(scope="module")
def rp(gpu_lib):
    import ringpop_amd
    return ringpop_amd


def _addr_table(S):
    addrs = S.addresses()
    bs = [a.encode() for a in addrs]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    return np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8), off


def _host_checksum(blob, off, st, inc):
    return oracle.lib().orc_view_checksum(oracle._ptr(blob), oracle._ptr(off), len(off) - 1,
                                          oracle._ptr(np.ascontiguousarray(st, dtype=np.uint8)),
                                          oracle._ptr(np.ascontiguousarray(inc, dtype=np.uint64)))


def _check_views(S, nodes, cs, blob, off):
    for v in nodes:
        st, inc = S.view(v)
        assert _host_checksum(blob, off, st, inc) == int(cs[v]), v
        rows = S.changes(v)
        info = S.info(v)
        if len(rows):
            a = rows[:, 0]
            assert len(np.unique(a)) == len(a), v                          # one key per address
            assert ((rows[:, 1] >= -1) & (rows[:, 1] <= info["max_pb"])).all(), v
            assert ((rows[:, 2] >= -1) & (rows[:, 2] < S.n)).all(), v       # source: a member or undefined
            assert np.array_equal(rows[:, 4], st[a]) and np.array_equal(rows[:, 5], inc[a].astype(np.int64)), v


def test_config4_full_size_invariants(rp):
    """Config 4 exactly as bench.py times it: 65,536 nodes, seed 2024, 656
    re-assertions per round, 85 rounds = the 60-round pre-roll + 5 warmup
    rounds + 20 timed rounds, so the state the headline is quoted on (steady
    log fill) is the state checked.  Sampled views' checksums are recomputed
    on the host after rounds 30, 65 and 85; dissemination invariants on the
    same nodes."""
    S = rp.Sim(N, 2024, churn_k=656)
    blob, off = _addr_table(S)
    rng = np.random.default_rng(4)
    done = 0
    for upto in (30, 65, 85):
        S.run(upto - done)
        done = upto
        S.sync()
        cs = S.checksums()
        nodes = sorted(set(rng.choice(N, size=24, replace=False).tolist()) | {0, N - 1})
        _check_views(S, nodes, cs, blob, off)
    c = S.counters()
    assert c["evaluated"] > 0 and c["applied"] > 0
    assert c["evaluated"] >= c["touched"] >= c["applied"]
    vc = S.view_counts()
    assert (vc[:, 1] == N).all() and (vc[:, 5] == N).all()  # full views, every member alive and in the ring
    print("compactions at 65,536 over 85 rounds: issue", c["compactions_issue"], "apply", c["compactions_apply"])
    S.close()


def test_checksum_paths_full_size(rp):
    """Every one of 65,536 checksums read after 30 rounds of config 4, once
    through one lane per view (k_checksums_pc) and once through one wave
    per view (k_checksums) on the same seeded state: identical, and 64 sampled
    views equal the oracle's restatement (orc_view_checksum over the view
    read back; lib/membership.js:41-93).  The lane path runs in the timed
    "observed" mode of bench.py (tick-cluster's every-node convergence check)."""
    got, hashed = {}, {}
    for mode, lane_min in (("lanes", 1), ("waves", 0xFFFFFFFF)):
        S = rp.Sim(N, 2024, churn_k=656, ck_lane_min=lane_min)
        try:
            S.run(30)
            S.sync()
            got[mode] = S.checksums()
            hashed[mode] = int(len(np.unique(got[mode])))
            if mode == "lanes":
                blob, off = _addr_table(S)
                nodes = sorted(set(np.random.default_rng(9).choice(N, size=62, replace=False).tolist()) | {0, N - 1})
                _check_views(S, nodes, got[mode], blob, off)
        finally:
            S.close()
    print("distinct checksums:", hashed)
    assert np.array_equal(got["lanes"], got["waves"])
    assert hashed["lanes"] > N // 2  # (config 4's views after a round: nearly all distinct)


def _trace(S, rounds):
    out = []
    for _ in range(rounds):
        o = S.round(churn=True)
        out.append((tuple(o[k] for k in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged")),
                    hashlib.sha256(S.checksums().tobytes()).hexdigest()))
    return out


def test_config4_full_size_shards_match_single(rp):
    """65,536 nodes on 1 shard and on 4 in-process shards (run one after the
    other: two do not fit in HBM together): identical counters and identical
    checksums of every node, every round."""
    a = rp.Sim(N, 7, churn_k=656)
    ta = _trace(a, 10)
    sa = {v: a.view(v)[1] for v in (0, 16383, 16384, 40000, N - 1)}
    a.close()
    b = rp.Sim(N, 7, churn_k=656, shards=4)
    tb = _trace(b, 10)
    for r, (x, y) in enumerate(zip(ta, tb)):
        assert x == y, r
    for v, inc in sa.items():
        assert np.array_equal(b.view(v)[1], inc), v
    b.close()


def test_config5_full_size_converges(rp):
    """Config 5: 6,554 of 65,536 nodes fail-stopped at round 0 and a seeded
    false-suspicion storm (0.1 % of live nodes per round for 20 rounds).
    Gossip until every live view is identical; then every failed node is
    faulty in every live view, every victim was refuted (no suspects), every
    live ring holds exactly the 58,982 live servers, and sampled checksums
    recompute on the host."""
    nf = -(-N // 10)
    dead = np.sort(np.random.default_rng(2024).choice(N, size=nf, replace=False))
    S = rp.Sim(N, 2024, churn_k=0, failures={0: dead.tolist()}, storm={"start": 0, "end": 20, "ppm": 1000})
    live = np.ones(N, dtype=bool)
    live[dead] = False
    done = None
    for r in range(150):
        st = S.round(churn=False)
        if st["converged"] and r >= 20:
            vc = S.view_counts()[live]
            if (vc[:, 3] == nf).all():
                done = r
                break
    assert done is not None, "config 5 did not converge in 150 rounds"
    vc = S.view_counts()[live]
    assert (vc[:, 1] == N - nf).all() and (vc[:, 2] == 0).all() and (vc[:, 3] == nf).all()
    assert (vc[:, 5] == N - nf).all()
    cs = S.checksums()
    assert len(np.unique(cs[live])) == 1
    blob, off = _addr_table(S)
    sample = np.flatnonzero(live)[:: (N - nf) // 16][:16]
    _check_views(S, sample.tolist(), cs, blob, off)
    S.close()


def _config5(rp, shards):
    nf = -(-N // 10)
    dead = np.sort(np.random.default_rng(2024).choice(N, size=nf, replace=False))
    kw = {"arena_entries": (N // shards) * 32768} if shards > 1 else {}  # (bench.py's sharded config-5 arena)
    S = rp.Sim(N, 2024, churn_k=0, failures={0: dead.tolist()}, storm={"start": 0, "end": 20, "ppm": 1000},
               shards=shards, **kw)
    live = np.ones(N, dtype=bool)
    live[dead] = False
    per = []
    for r in range(150):
        st = S.round(churn=False)
        per.append(tuple(st[k] for k in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged")))
        if st["converged"] and r >= 20:
            vc = S.view_counts()[live]
            if (vc[:, 3] == nf).all():
                break
    cs = S.checksums()
    probe = [int(x) for x in np.flatnonzero(live)[:: (N - nf) // 8][:8]]
    views = {v: (S.view(v)[0].copy(), S.view(v)[1].copy(), S.members(v).copy(), S.changes(v).copy()) for v in probe}
    vc = S.view_counts()
    S.close()
    return per, cs, views, vc, live


def test_config5_full_size_shards_match_single(rp):
    """Config 5 at 65,536 nodes on 1 shard, then (the same cluster rebuilt) on
    4 in-process shards: the mass failure, the false-suspicion storm, the
    ping-req waves, suspicion timeouts and refutes cross the shards (16-byte
    escapes, the local-origin all-gather, fullSync expansion).  Identical
    per-round counters through convergence, identical checksums of every
    live node and identical sampled views, member orders and dissemination
    tables at the end."""
    pa, ca, va, vca, live = _config5(rp, 1)
    pb, cb, vb, vcb, _ = _config5(rp, 4)
    assert len(pa) == len(pb), (len(pa), len(pb))
    for r, (x, y) in enumerate(zip(pa, pb)):
        assert x == y, r
    assert np.array_equal(ca[live], cb[live])
    assert np.array_equal(vca[live], vcb[live])
    for v in va:
        for a, b in zip(va[v], vb[v]):
            assert np.array_equal(a, b), v


def test_oracle_fixture_n8192(rp, golden):
    """N = 8,192 against the C oracle (fixture from oracle/gen_large_fixture.py):
    churn, a 10 % fail-stop at round 5 and a false-suspicion storm, 48 rounds --
    per-round counters and every node's checksum, then sampled nodes' views,
    member orders and dissemination tables."""
    g = golden("sim_oracle_n8192.json.gz")
    cfg = g["config"]
    dead = np.array(g["failed"])
    S = rp.Sim(cfg["n"], cfg["seed"], churn_k=cfg["churnK"], failures={cfg["failRound"]: g["failed"]},
               storm=cfg["storm"])
    for r, want in enumerate(g["rounds"]):
        o = S.round(churn=r < cfg["churnRounds"])
        for k in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert o[k] == want[k], (r, k, o[k], want[k])
        cs = S.checksums()
        if r >= cfg["failRound"]:
            cs[dead] = 0
        assert hashlib.sha256(cs.tobytes()).hexdigest() == want["checksums_sha256"], r
    cs = S.checksums()
    cs[dead] = 0
    assert cs.tolist() == g["final"]["checksums"]

    def digest(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    for v, d in g["final"]["nodes"].items():
        v = int(v)
        st, inc = S.view(v)
        assert digest(st.astype(np.uint8)) == d["view_status"] and digest(inc.astype(np.uint64)) == d["view_inc"], v
        assert digest(np.asarray(S.members(v), dtype=np.int32)) == d["members"], v
        assert digest(np.asarray(S.changes(v), dtype=np.int64).reshape(-1, 6)) == d["changes"], v
        info = S.info(v)
        assert {k: info[k] for k in d["info"]} == d["info"], v
    cnt = S.counters()
    print("prefix packs", cnt["prefix_packs"], "same-view issues", cnt["same_view_issues"])
    assert cnt["prefix_packs"] > 0 and cnt["same_view_issues"] > 0  # both fired under the oracle's fixture
    S.close()


def test_config3_string_keys_10k_servers(rp):
    """k_lookup_keys on decimal u64 string keys (config 3's key shape) against
    a 10,000-server x 100-point ring: 2,000,000 keys through the C ABI and the
    device key generator, every owner against the oracle's restatement."""
    names = [f"10.{i >> 16 & 255}.{i >> 8 & 255}.{i & 255}:{3000 + i % 7}" for i in range(10_000)]
    ring = rp.HashRing()
    assert ring.addRemoveServers(names, None)
    ph, po = oracle.ring_points_add_only(names)
    h, o = ring.points()
    assert np.array_equal(h, ph) and np.array_equal(o, po)
    keys = oracle.lookup_keys(99, np.arange(2_000_000))
    want = oracle.ring_lookup_points(ph, po, oracle.farmhash32_batch(keys))
    got = ring.lookup_indices(keys)
    assert np.array_equal(got, want)
    # the same keys generated on the device (rp_ring_make_keys_device), resident in HBM
    assert np.array_equal(_lookup_device_keys(ring, 99, len(keys)), want)
    ring.close()


def _lookup_device_keys(ring, seed, n):
    """rp_ring_make_keys_device + rp_ring_lookup_batch_device (the bench's
    path): keys and owners resident on the device."""
    import ctypes

    from ringpop_amd import hiprt
    from ringpop_amd._lib import check, lib
    L = lib()
    d_bytes, d_off, total = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    check(L.rp_ring_make_keys_device(ring._h, seed, n, ctypes.byref(d_bytes), ctypes.byref(d_off),
                                     ctypes.byref(total)))
    own = hiprt.DeviceArray(n, np.int32)
    check(L.rp_ring_lookup_batch_device(ring._h, d_bytes, d_off, n, own.ptr, None))
    out = own.numpy()
    own.free()
    return out
