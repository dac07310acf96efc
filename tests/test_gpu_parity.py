"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden fixtures.  Integer/byte work: bit-exact everywhere."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rp(gpu_lib):
    import ringpop_amd
    return ringpop_amd


def test_farmhash_vectors(rp, golden):
    g = golden("farmhash_vectors.json")
    assert rp.hash32_batch(g["strings"]).tolist() == g["hash32"]
    assert rp.hash32("") == 0xDC56D17A


def test_farmhash_random_lengths(rp):
    rng = np.random.default_rng(1)
    strs = [bytes(rng.integers(0, 256, size=int(l), dtype=np.uint8)) for l in rng.integers(0, 300, size=3000)]
    assert np.array_equal(rp.hash32_batch(strs), oracle.farmhash32_batch(strs))


def test_farmhash_long_and_scalar(rp):
    """Strings of HASH_LONG_MIN (1,024) bytes and more are hashed one wave each
    (rp_whash.h: LDS-staged spans, any start alignment inside a batch); scalar
    rp_hash32 calls up to 3,072 bytes take the kernel-argument path, longer
    ones the wave path."""
    rng = np.random.default_rng(2)
    lens = [1023, 1024, 1025, 3839, 3840, 3841, 3860, 7681, 20000, 65537] + list(rng.integers(1000, 40000, size=30))
    strs = [bytes(rng.integers(0, 256, size=int(l), dtype=np.uint8)) for l in lens]
    mixed = [b"", b"x" * 7] + strs + [b"10.0.0.1:3000"]  # short and long in one batch: odd byte offsets
    assert np.array_equal(rp.hash32_batch(mixed), oracle.farmhash32_batch(mixed))
    for s in [b"", b"a", b"12345", b"x" * 24, b"y" * 25] + strs[:12] + [bytes(range(256)) * 12]:
        assert rp.hash32(s) == int(oracle.farmhash32_batch([s])[0]), len(s)
    big = b";".join(b"10.%d.%d.1:3000alive1434401518824" % (i // 250, i % 250) for i in range(65536))
    assert rp.hash32(big) == int(oracle.farmhash32_batch([big])[0])


def test_ring_scalar_lookup_matches_batch(rp):
    ring = rp.HashRing()
    ring.addRemoveServers([f"10.{i // 250}.{i % 250}.1:3000" for i in range(1000)], None)
    rng = np.random.default_rng(3)
    keys = [str(x) for x in rng.integers(0, 10**12, size=500)] + ["", "k" * 3000, "k" * 3100]
    batch = [ring.server_name(int(o)) for o in ring.lookup_batch(keys)]
    assert [ring.lookup(k) for k in keys] == batch


def test_ring_farmhash_fixture(rp, golden):
    g = golden("ring_farmhash.json")
    ring = rp.HashRing()
    assert ring.addRemoveServers(g["servers"], None)
    owners = [ring.server_name(int(o)) for o in ring.lookup_batch(g["keys"])]
    assert owners == g["owners"]
    # test/ring-test.js:66-80: lookup(server + '0') === server
    for s in g["servers"][:50]:
        assert ring.lookup(s + "0") == s
    ring.addRemoveServers(None, g["removed"])
    assert ring.getServerCount() == g["server_count"]
    assert [ring.server_name(int(o)) for o in ring.lookup_batch(g["keys"])] == g["owners_after_remove"]
    assert ring.checksum == g["checksum_after_remove"]
    assert [ring.lookupN(k, 3) for k in g["keys"][:200]] == g["lookupN3_after_remove"]


def test_ring_collision_history(rp, golden):
    """Forced replica-hash collisions through the hashFunc seam (lib/ring.js:29)."""
    g = golden("ring_collisions.json")
    table = g["table"]

    def hf(s):  # replica names via the table, probe keys "key:<n>" -> n
        if s in table:
            return table[s]
        return int(s[4:]) if s[4:].isdigit() else 0

    ring = rp.HashRing(replica_points=g["replica_points"], hash_func=hf)
    for step in g["steps"]:
        assert ring.addRemoveServers(step["add"], step["remove"]) == step["changed"]
        h, o = ring.points()
        assert [[int(a), ring.server_name(int(b))] for a, b in zip(h, o)] == step["points"]
        got = [ring.server_name(int(x)) for x in ring.lookup_hashes([hf(p) for p in g["probes"]])]
        assert got == step["lookups"]
        assert [ring.lookupN(p, 3) for p in g["probes"][:40]] == step["lookupN"]


def views_of(cfg):
    """cfg["views"][i][j] = [status, incarnation] -> (status, inc) arrays, or None"""
    if "views" not in cfg:
        return None
    v = np.array(cfg["views"], dtype=np.int64)
    return v[:, :, 0], v[:, :, 1]


def _gpu_matches_case(rp, case, check_final=True, shards=1, ck_lane_min=0):
    cfg = case["config"]
    fail = {int(k): v for k, v in cfg.get("failures", {}).items()}
    S = rp.Sim(cfg["n"], cfg["seed"], churn_k=cfg.get("churnK"), failures=fail, partition=cfg.get("partition"),
               storm=cfg.get("storm"), addresses=cfg.get("addresses"), views=views_of(cfg), shards=shards,
               joins=[tuple(e) for e in cfg.get("joins", [])] or None, ck_lane_min=ck_lane_min)
    for r, jr in enumerate(case["rounds"]):
        o = S.round(churn=r < cfg["churnRounds"])
        for k, jk in (("evaluated", "evaluated"), ("applied", "applied"), ("full_syncs", "fullSyncs"),
                      ("messages", "messages"), ("waves", "waves")):
            assert o[k] == jr[jk], (r, k, o[k], jr[jk])
        got = S.checksums().tolist()
        assert [None if w is None else x for x, w in zip(got, jr["checksums"])] == jr["checksums"], r
        assert bool(o["converged"]) == jr["converged"], r
    if check_final and "final" in case:
        for v, f in enumerate(case["final"]):
            st, inc = S.view(v)
            for a, e in enumerate(f["view"]):
                assert (int(st[a]), int(inc[a])) == ((0, 0) if e is None else tuple(e)), (v, a)
            assert S.members(v).tolist() == f["members"], v
            assert S.changes(v).tolist() == f["changes"], v
            info = S.info(v)
            assert info["max_pb"] == f["maxPiggyback"] and info["ring_servers"] == f["ringServers"], v
            if f["ringChecksum"] is not None:  # (an empty ring never computed one: a node that never joined)
                assert info["ring_checksum"] == f["ringChecksum"], v
            assert info["iter_index"] == f["iterIndex"] and info["iter_round"] == f["iterRound"], v
            assert (info["rng"] & (2**64 - 1)) == int(f["rng"]), v
    return S


@pytest.mark.parametrize("idx", [0, 1, 2, 3, 4])
def test_sim_small_against_reference(rp, golden, idx):
    # 0-1 churn (1 wraps the iterator and reshuffles); 2 and 4 fail-stops
    # (ping-req, suspicion timeouts, faulty ring removals); 3 a partition
    # (full syncs after it heals)
    _gpu_matches_case(rp, golden("sim_small.json.gz")["cases"][idx])


def test_sim_medium_failures_partition_against_reference(rp, golden):
    case = golden("sim_medium.json.gz")["cases"][1]
    S = _gpu_matches_case(rp, case, check_final=False)
    assert S.checksums().tolist() == case["final_checksums"]


def test_sim_n256_against_reference(rp, golden):
    case = golden("sim_medium.json.gz")["cases"][0]
    S = _gpu_matches_case(rp, case, check_final=False)
    assert S.checksums().tolist() == case["final_checksums"]


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_sim_storm_against_reference(rp, golden, idx):
    """Config 5's false-suspicion storm: accusers' makeSuspect (lib/membership.js:
    154-156) refuted by the victims (:244-254), alone and with fail-stops."""
    case = golden("sim_storm.json.gz")["cases"][idx]
    S = _gpu_matches_case(rp, case, check_final="final" in case)
    if "final_checksums" in case:
        got = S.checksums().tolist()
        assert [None if w is None else x for x, w in zip(got, case["final_checksums"])] == case["final_checksums"]


@pytest.mark.parametrize("name,idx,shards", [
    ("sim_small.json.gz", 0, 1), ("sim_small.json.gz", 1, 1), ("sim_small.json.gz", 2, 1), ("sim_small.json.gz", 3, 1),
    ("sim_small.json.gz", 4, 1), ("sim_medium.json.gz", 0, 1), ("sim_medium.json.gz", 1, 2),
    ("sim_storm.json.gz", 0, 1), ("sim_storm.json.gz", 2, 4), ("sim_views.json.gz", 0, 1), ("sim_views.json.gz", 1, 1),
    ("sim_views.json.gz", 2, 2), ("sim_views.json.gz", 3, 1), ("sim_join.json.gz", 0, 1), ("sim_join.json.gz", 1, 1),
    ("sim_join.json.gz", 2, 2), ("sim_join.json.gz", 3, 4)])
def test_sim_checksums_lane_per_view_against_reference(rp, golden, name, idx, shards):
    """Every checksum through k_checksums_pc (ck_lane_min = 1: one lane
    per view, the view's length from SimDev::slen): the senders' checksums the
    protocol reads each round and every node's checksum read after it, on the
    reference's fixtures -- churn, fail-stops, partitions, storms, arbitrary
    addresses and per-node views (absent members, every status) and joins
    (views growing from empty) -- on 1-4 shards (lib/membership.js:41-93)."""
    case = golden(name)["cases"][idx]
    _gpu_matches_case(rp, case, check_final=False, shards=shards, ck_lane_min=1)


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_sim_views_against_reference(rp, golden, idx):
    """Arbitrary clusters (rp_sim_load_addresses, rp_sim_set_views): loaded
    4-32-byte addresses and per-node bootstrap views (suspects with timers due
    at round 0, faulty and leave members outside the ring) against the
    reference bootstrapped from the same views."""
    case = golden("sim_views.json.gz")["cases"][idx]
    S = _gpu_matches_case(rp, case, check_final="final" in case)
    if "final_checksums" in case:
        got = S.checksums().tolist()
        assert [None if w is None else x for x, w in zip(got, case["final_checksums"])] == case["final_checksums"]
    if case["config"].get("addresses"):
        assert [S.address(i) for i in range(S.n)] == case["config"]["addresses"]


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_sim_join_against_reference(rp, golden, idx):
    """The join path (rp_sim_join): nodes outside the cluster join through
    seeds -- makeAlive(self), handleJoin's makeAlive + fullSync replies,
    mergeJoinResponses, set(), shuffle() -- and gossip splices them into every
    view at getJoinPosition (the device's absent-member merge)."""
    case = golden("sim_join.json.gz")["cases"][idx]
    S = _gpu_matches_case(rp, case, check_final="final" in case)
    if "final_checksums" in case:
        assert S.checksums().tolist() == case["final_checksums"]


@pytest.mark.parametrize("idx,shards", [(1, 2), (1, 4), (3, 4), (2, 8)])
def test_sim_join_sharded_against_reference(rp, golden, idx, shards):
    case = golden("sim_join.json.gz")["cases"][idx]
    S = _gpu_matches_case(rp, case, check_final="final" in case, shards=shards)
    if "final_checksums" in case:
        assert S.checksums().tolist() == case["final_checksums"]


def test_sim_join_against_oracle(rp):
    """512 nodes: 64 members, the rest join 32 per round through 3 seeds, with
    churn and fail-stops; device vs oracle every round and final views."""
    n, seed = 512, 51
    r = np.random.default_rng(9)
    ids = r.permutation(n).tolist()
    members, joins, rnd = ids[:64], [], 0
    failed = {3: [members[5]], 6: [ids[100]]}
    for q in range(64, n, 32):
        batch = ids[q:q + 32]
        for j in batch:
            joins.append((rnd, j, [int(x) for x in r.choice(members, size=3, replace=False)]))
        members = members + batch
        rnd += 1
    members_dead = {m for v in failed.values() for m in v}
    joins = [(a, j, [x for x in sd if x not in members_dead]) for a, j, sd in joins]
    g = rp.Sim(n, seed, churn_k=3, joins=joins, failures=failed)
    c = oracle.Sim(n, seed, churn_k=3, joins=joins, failures=failed)
    for rr in range(60):
        a, b = g.round(churn=rr < 30), c.round(churn=rr < 30)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert a[key] == b[key], (rr, key, a[key], b[key])
        gc = g.checksums().tolist()
        assert gc == [x if x is not None else gc[i] for i, x in enumerate(c.checksums())], rr
    for v in range(0, n, 23):
        assert g.members(v).tolist() == c.members(v).tolist(), v
        assert g.changes(v).tolist() == c.changes(v).tolist(), v
        sg, ig = g.view(v)
        sc, ic = c.view(v)
        assert np.array_equal(sg, sc) and np.array_equal(ig, ic), v


@pytest.mark.parametrize("shards", [2, 4])
def test_sim_views_sharded_against_reference(rp, golden, shards):
    _gpu_matches_case(rp, golden("sim_views.json.gz")["cases"][1], shards=shards)


def test_sim_views_against_oracle(rp):
    """Random bootstrap views at n = 512 on loaded addresses, device vs oracle."""
    n, seed = 512, 31
    r = np.random.default_rng(5)
    addrs = sorted({f"{r.integers(1, 999999)}.{r.integers(0, 256)}.{r.integers(0, 256)}.{i}:{r.integers(1, 65536)}"
                    for i in range(n)})
    assert len(addrs) == n
    base_st = r.choice([1, 1, 1, 1, 1, 1, 2, 3, 4], size=n)
    base_inc = 1434401518824 + np.arange(n) + 1000 * r.integers(0, 4, size=n)
    st = np.tile(base_st, (n, 1)).astype(np.int32)
    inc = np.tile(base_inc, (n, 1)).astype(np.int64)
    noise = r.random((n, n)) < 0.05
    st[noise] = r.choice([1, 2, 3, 4], size=int(noise.sum()))
    inc[noise] += 1000 * r.integers(0, 2, size=int(noise.sum()))
    st[np.arange(n), np.arange(n)] = 1
    g = rp.Sim(n, seed, churn_k=3, addresses=addrs, views=(st, inc), failures={2: [7, 300]})
    c = oracle.Sim(n, seed, churn_k=3, addresses=addrs, views=(st, inc), failures={2: [7, 300]})
    for rnd in range(60):
        go, co = g.round(churn=rnd < 20), c.round(churn=rnd < 20)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves"):
            assert go[key] == co[key], (rnd, key)
        gc = g.checksums().tolist()
        assert gc == [x if x is not None else gc[i] for i, x in enumerate(c.checksums())], rnd
    for v in range(0, n, 37):
        gs, gi = g.view(v)
        cs, ci = c.view(v)
        assert np.array_equal(gs, cs) and np.array_equal(gi, ci), v
        assert g.members(v).tolist() == c.members(v).tolist(), v
        assert g.changes(v).tolist() == c.changes(v).tolist(), v


def test_sim_views_argument_checks(rp):
    from ringpop_amd._lib import RingpopError
    S = rp.Sim(8, 1)
    with pytest.raises(RingpopError):
        S.load_addresses([f"1.1.1.{i}:1" for i in range(8)][::-1])  # not sorted
    with pytest.raises(RingpopError):
        S.load_addresses(["1.1.1.1:" + "9" * 30] + [f"2.2.2.{i}:1" for i in range(7)])  # 39 bytes
    st = np.ones((8, 8), dtype=np.int32)
    inc = np.full((8, 8), 5, dtype=np.int64)
    st[3, 3] = 2
    with pytest.raises(RingpopError):
        S.set_views(st, inc)  # own entry not alive
    st[3, 3] = 1
    st[1, 2] = 5
    with pytest.raises(RingpopError):
        S.set_views(st, inc)  # no such status
    st[1, 2] = 0
    S.set_views(st, inc)  # an absent member: a partial view
    assert 2 not in S.members(1).tolist() and len(S.members(1)) == 7
    with pytest.raises(RingpopError):
        S.load_addresses([f"1.1.1.{i}:1" for i in range(8)])  # would rebuild full views over set_views
    assert 2 not in S.members(1).tolist()
    J = rp.Sim(8, 1)
    J.join([(7, 2, [0])])
    with pytest.raises(RingpopError):
        J.load_addresses([f"1.1.1.{i}:1" for i in range(8)])  # would drop the join schedule
    J.close()
    S.round()
    with pytest.raises(RingpopError):
        S.load_addresses([f"1.1.1.{i}:1" for i in range(8)])  # after the first round
    S.close()


@pytest.mark.parametrize("n,seed,k,rounds,fail,storm", [
    (300, 6, 3, 70, {0: [5, 6, 7, 100, 250]}, {"start": 0, "end": 40, "ppm": 10000}),
    (500, 2, 0, 60, None, {"start": 3, "end": 30, "ppm": 1000}),
    (256, 3, 2, 80, {0: list(range(0, 256, 10))}, {"start": 0, "end": 50, "ppm": 30000})])
def test_sim_storm_against_oracle(rp, n, seed, k, rounds, fail, storm):
    g = rp.Sim(n, seed, churn_k=k, failures=fail, storm=storm)
    c = oracle.Sim(n, seed, churn_k=k, failures=fail, storm=storm)
    for r in range(rounds):
        a = g.round(churn=r < rounds // 2)
        b = c.round(churn=r < rounds // 2)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert a[key] == b[key], (r, key, a[key], b[key])
        got = g.checksums().tolist()
        assert [x if w is not None else None for x, w in zip(got, c.checksums())] == c.checksums(), r
    for v in range(0, n, max(1, n // 13)):
        if c.info(v)["dead"]:
            continue
        assert g.changes(v).tolist() == c.changes(v).tolist(), v
        assert np.array_equal(g.view(v)[1], c.view(v)[1]) and np.array_equal(g.view(v)[0], c.view(v)[0]), v
        assert g.members(v).tolist() == c.members(v).tolist(), v


def test_sim_config2_n1024_against_reference(rp, golden):
    case = golden("sim_config2_n1024.json.gz")["cases"][0]
    S = _gpu_matches_case(rp, case, check_final=False)
    assert case["convergedAt"] == len(case["rounds"]) - 1
    cnt = S.counters()
    # (at 1,024 nodes a log ring of n slots never holds a window the default
    # packing threshold can shrink: test_sim_prefix_packing_against_oracle
    # forces it, the 8,192-node fixture runs it at the default)
    print("prefix packs", cnt["prefix_packs"], "same-view issues", cnt["same_view_issues"])
    assert cnt["same_view_issues"] > 0


@pytest.mark.parametrize("n,seed,k,rounds,fail,part,win", [
    (100, 3, 3, 40, None, None, 0), (500, 11, 5, 30, None, None, 0), (33, 5, 1, 120, None, None, 0),
    (300, 4, 3, 60, {0: [1, 50, 77], 5: [200]}, None, 0),
    (120, 8, 2, 70, None, {"start": 2, "end": 30, "split": 50}, 0),
    (200, 13, 2, 80, {1: list(range(0, 200, 10))}, {"start": 10, "end": 40, "split": 120}, 0),
    # tiny seen-origin windows: the bitset wraps every few rounds (and every
    # round when more ids than the window are allocated per round)
    (100, 3, 3, 40, None, None, 32), (300, 4, 3, 60, {0: [1, 50, 77], 5: [200]}, None, 64),
    (500, 11, 40, 30, None, None, 32), (256, 21, 9, 50, None, None, 128)])
def test_sim_against_oracle(rp, n, seed, k, rounds, fail, part, win):
    g = rp.Sim(n, seed, churn_k=k, failures=fail, partition=part, seen_window=win)
    c = oracle.Sim(n, seed, churn_k=k, failures=fail, partition=part)
    for r in range(rounds):
        a = g.round(churn=r < rounds * 2 // 3)
        b = c.round(churn=r < rounds * 2 // 3)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert a[key] == b[key], (r, key, a[key], b[key])
        assert g.checksums().tolist() == [x if x is not None else g.checksums()[i] for i, x in enumerate(c.checksums())], r
    for v in range(0, n, max(1, n // 17)):
        assert g.changes(v).tolist() == c.changes(v).tolist()
        sg, ig = g.view(v)
        sc, ic = c.view(v)
        assert np.array_equal(sg, sc) and np.array_equal(ig, ic)
        assert g.members(v).tolist() == c.members(v).tolist()


@pytest.mark.parametrize("n,seed,k,rounds,fail,storm,part,compact,shards", [
    (256, 5, 6, 60, {0: [3, 40, 41, 200]}, {"start": 0, "end": 40, "ppm": 20000}, None, (1, 16), 1),
    (256, 5, 6, 60, {0: [3, 40, 41, 200]}, {"start": 0, "end": 40, "ppm": 20000}, None, (1, 16), 4),
    (300, 9, 4, 50, None, None, {"start": 5, "end": 30, "split": 120}, (0, 1), 1),
    (192, 2, 9, 70, {10: list(range(0, 192, 16))}, {"start": 2, "end": 60, "ppm": 10000}, None, (1, 4), 4)])
def test_sim_issue_compaction_against_oracle(rp, n, seed, k, rounds, fail, storm, part, compact, shards):
    """Issue-time log compaction (wg_issue: span > compact_mul x live keys +
    compact_add) forced with tiny thresholds, so that it fires many times
    under churn, fail-stops, false-suspicion storms and partitions, on one and
    four shards.  At the default thresholds (4x + 8,192) it cannot fire below
    ~8k nodes, where the apply-time trigger always comes first.  Key order,
    piggyback counts, deletions and sources (lib/dissemination.js:138-182)
    must stay the oracle's, which has no compaction at all."""
    g = rp.Sim(n, seed, churn_k=k, failures=fail, storm=storm, partition=part, compact=compact, shards=shards)
    c = oracle.Sim(n, seed, churn_k=k, failures=fail, storm=storm, partition=part)
    for r in range(rounds):
        a = g.round(churn=r < rounds * 2 // 3)
        b = c.round(churn=r < rounds * 2 // 3)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert a[key] == b[key], (r, key, a[key], b[key])
        got = g.checksums().tolist()
        assert [x if w is not None else None for x, w in zip(got, c.checksums())] == c.checksums(), r
        if r % 10 == 9:
            for v in range(r % 7, n, max(1, n // 11)):
                if not c.info(v)["dead"]:
                    assert g.changes(v).tolist() == c.changes(v).tolist(), (r, v)
    for v in range(0, n, max(1, n // 13)):
        if c.info(v)["dead"]:
            continue
        assert g.changes(v).tolist() == c.changes(v).tolist(), v
        assert np.array_equal(g.view(v)[1], c.view(v)[1]) and np.array_equal(g.view(v)[0], c.view(v)[0]), v
        assert g.members(v).tolist() == c.members(v).tolist(), v
    cnt = g.counters()
    print("compactions: issue", cnt["compactions_issue"], "apply", cnt["compactions_apply"])
    assert cnt["compactions_issue"] > n, cnt["compactions_issue"]  # fired many times (1,971 at 256 nodes, (1, 16))
    g.close()


@pytest.mark.parametrize("n,seed,k,rounds,fail,storm,part,pmin,compact,shards", [
    (256, 5, 6, 60, {0: [3, 40, 41, 200]}, {"start": 0, "end": 40, "ppm": 20000}, None, 1, None, 1),
    (256, 5, 6, 60, {0: [3, 40, 41, 200]}, {"start": 0, "end": 40, "ppm": 20000}, None, 8, None, 4),
    (300, 9, 4, 50, None, None, {"start": 5, "end": 30, "split": 120}, 32, None, 1),
    (192, 2, 9, 70, {10: list(range(0, 192, 16))}, {"start": 2, "end": 60, "ppm": 10000}, None, 1, (1, 4), 4),
    (512, 7, 12, 60, {20: [1, 2, 3, 300]}, None, {"start": 30, "end": 45, "split": 200}, 8, (1, 16), 1)])
def test_sim_prefix_packing_against_oracle(rp, n, seed, k, rounds, fail, storm, part, pmin, compact, shards):
    """The issue's head packing (wg_pack_prefix: after an issue the live
    entries of the window's first groups move, in order, to the end of that
    prefix and the head jumps past the dead part) forced with tiny thresholds
    (rp_sim_config.prefix_min; the default 512 cannot fire while a log ring
    holds n <= 512 slots), alone and together with forced compaction, under
    churn, fail-stops, storms and a partition on one and four shards.  An
    overwritten key keeps its slot (lib/dissemination.js:125-127), so key
    order, counts and sources (:138-182) must stay the oracle's, which has
    neither packing nor compaction.  The same-view single-entry issue
    (identical views: only the destination's own entry is written) fires too."""
    g = rp.Sim(n, seed, churn_k=k, failures=fail, storm=storm, partition=part, compact=compact, shards=shards,
               prefix_min=pmin)
    c = oracle.Sim(n, seed, churn_k=k, failures=fail, storm=storm, partition=part)
    for r in range(rounds):
        a = g.round(churn=r < rounds * 2 // 3)
        b = c.round(churn=r < rounds * 2 // 3)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert a[key] == b[key], (r, key, a[key], b[key])
        got = g.checksums().tolist()
        assert [x if w is not None else None for x, w in zip(got, c.checksums())] == c.checksums(), r
        if r % 10 == 9:
            for v in range(r % 7, n, max(1, n // 11)):
                if not c.info(v)["dead"]:
                    assert g.changes(v).tolist() == c.changes(v).tolist(), (r, v)
    for v in range(0, n, max(1, n // 13)):
        if c.info(v)["dead"]:
            continue
        assert g.changes(v).tolist() == c.changes(v).tolist(), v
        assert np.array_equal(g.view(v)[1], c.view(v)[1]) and np.array_equal(g.view(v)[0], c.view(v)[0]), v
        assert g.members(v).tolist() == c.members(v).tolist(), v
    cnt = g.counters()
    print("prefix packs", cnt["prefix_packs"], "same-view issues", cnt["same_view_issues"],
          "compactions", cnt["compactions_issue"])
    assert cnt["prefix_packs"] > n, cnt["prefix_packs"]
    assert cnt["same_view_issues"] > 0
    if compact:
        assert cnt["compactions_issue"] > 0
    g.close()


def test_sim_origin_rings_wrap_against_oracle(rp):
    """Update-origin ids are reused: with a 512-slot origin table
    the makeAlive ring (256 slots) and the local suspect/faulty ring (128
    slots) wrap many times over 300 rounds of churn, false suspicions and a
    fail-stop; every round still equals the oracle, which has no table."""
    n, seed, k = 64, 3, 3
    fail = {10: [5], 120: [40]}
    storm = {"start": 0, "end": 300, "ppm": 20000}
    g = rp.Sim(n, seed, churn_k=k, failures=fail, storm=storm, origin_slots=512)
    c = oracle.Sim(n, seed, churn_k=k, failures=fail, storm=storm)
    for r in range(300):
        a = g.round(churn=r < 280)
        b = c.round(churn=r < 280)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert a[key] == b[key], (r, key, a[key], b[key])
        got = g.checksums().tolist()
        assert [x if w is not None else None for x, w in zip(got, c.checksums())] == c.checksums(), r
    for v in range(0, n, 7):
        if not c.info(v)["dead"]:
            assert g.changes(v).tolist() == c.changes(v).tolist(), v


def test_sim_ring_lookup_matches_oracle(rp):
    n = 300
    g = rp.Sim(n, 9, churn_k=3)
    c = oracle.Sim(n, 9, churn_k=3)
    g.round(); c.round()
    keys = np.random.default_rng(5).integers(0, 2**32, size=2000, dtype=np.uint64).astype(np.uint32)
    for v in (0, 17, 299):
        assert g.ring_lookup(v, keys).tolist() == [c.ring_lookup(v, int(h)) for h in keys]


@pytest.mark.parametrize("n,seed,shift,fail,part", [
    (200, 3, 18, {2: [5, 9, 17, 40, 41, 42, 43, 44, 45, 46]}, None),
    (256, 7, 20, {0: list(range(3, 256, 9))}, {"start": 4, "end": 30, "split": 100}),
    (150, 1, 22, {1: list(range(0, 150, 4))}, None)])
def test_sim_forced_ring_collisions(rp, n, seed, shift, fail, part):
    """Replica hashes truncated to 32 - shift bits: most replica points collide,
    so every faulty removal erases other servers' points and re-adds contend for
    them (lib/rbtree.js:112-117,152); views must match the oracle's rbtree model,
    including ring lookups in each view."""
    g = rp.Sim(n, seed, churn_k=3, failures=fail, partition=part, replica_hash_shift=shift)
    c = oracle.Sim(n, seed, churn_k=3, failures=fail, partition=part, replica_hash_shift=shift)
    keys = np.random.default_rng(seed).integers(0, 2**32, size=500, dtype=np.uint64).astype(np.uint32)
    for r in range(70):
        a = g.round(churn=r < 40)
        b = c.round(churn=r < 40)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert a[key] == b[key], (r, key, a[key], b[key])
        if r % 10 == 9:
            for v in range(1, n, n // 7):
                if c.info(v)["dead"]:
                    continue
                assert g.info(v)["ring_servers"] == c.info(v)["ring_servers"], (r, v)
                assert g.ring_lookup(v, keys).tolist() == [c.ring_lookup(v, int(h)) for h in keys], (r, v)


def _grouped(keys, owners):
    """_.groupBy(keys, lookup) built from the reference fixture's owners."""
    out = {}
    for k, o in zip(keys, owners):
        out.setdefault(o, []).append(k)
    return out


def test_group_by_owner_fixture(rp, golden):
    """handleOrProxyAll grouping (index.js:636-645) on the reference ring fixture."""
    g = golden("ring_farmhash.json")
    ring = rp.HashRing()
    assert ring.groupByOwner(g["keys"][:10]) == {None: g["keys"][:10]}  # empty ring: the null group
    assert ring.groupByOwner([]) == {}
    ring.addRemoveServers(g["servers"], None)
    got = ring.groupByOwner(g["keys"])
    want = _grouped(g["keys"], g["owners"])
    assert list(got) == list(want)  # dest order: first appearance
    assert got == want
    ring.addRemoveServers(None, g["removed"])
    assert ring.groupByOwner(g["keys"]) == _grouped(g["keys"], g["owners_after_remove"])
    ring.close()


def test_group_by_owner_empty_ring(rp):
    ring = rp.HashRing()
    keys = [f"k{i}" for i in range(100)]
    assert ring.groupByOwner(keys) == {None: keys}
    d, off, idx = ring.group_indices(keys)
    assert d.tolist() == [-1] and off.tolist() == [0, 100] and idx.tolist() == list(range(100))
    ring.close()


# (the grouping's radix sort: 1 pass for <= 256 groups, 2 up to 65,536, 3
# beyond; owner counts above 12,288 take the global-atomic path)
@pytest.mark.parametrize("nserv,nkeys", [(1, 1000), (3, 1), (1000, 300_000), (10_000, 2_000_000),
                                         (40_000, 3_000_000)])
def test_group_by_owner_large_against_oracle(rp, nserv, nkeys):
    names = [f"10.{i >> 16 & 255}.{i >> 8 & 255}.{i & 255}:{3000 + i % 7}" for i in range(nserv)]
    ring = rp.HashRing()
    ring.addRemoveServers(names, None)
    ph, po = oracle.ring_points_add_only(names)
    kh = np.random.default_rng(nkeys).integers(0, 2**32, size=nkeys, dtype=np.uint64).astype(np.uint32)
    want = oracle.group_by_owner_np(oracle.ring_lookup_points(ph, po, kh))
    n = len(kh)
    import ctypes
    from ringpop_amd._lib import check, lib, ptr
    dests = np.zeros(n, np.int32)
    goff = np.zeros(n + 1, np.uint32)
    kidx = np.zeros(n, np.uint32)
    ng = ctypes.c_size_t(0)
    check(lib().rp_ring_group_hashes(ring._h, ptr(kh), n, ptr(dests), ptr(goff), ptr(kidx), ctypes.byref(ng)))
    g = ng.value
    assert np.array_equal(dests[:g], want[0])
    assert np.array_equal(goff[: g + 1], want[1])
    assert np.array_equal(kidx, want[2])
    ring.close()


def test_group_by_owner_custom_hash_collisions(rp):
    """hashFunc seam (lib/ring.js:29): a coarse hash makes replicas collide and
    many keys share points; grouping follows the device lookups exactly."""
    def hf(s):
        return oracle.farmhash32(s) & 0xFFF00000
    names = [f"s{i}" for i in range(40)]
    ring = rp.HashRing(replica_points=10, hash_func=hf)
    ring.addRemoveServers(names, names[:7])
    keys = [f"key{i}" for i in range(5000)]
    owners = ring.lookup_hashes(np.array([hf(k) for k in keys], dtype=np.uint32))
    want = oracle.group_by_owner(owners)
    d, off, idx = ring.group_indices(keys)
    assert np.array_equal(d, want[0]) and np.array_equal(off, want[1]) and np.array_equal(idx, want[2])
    ring.close()


def test_fingerprint_path_near_collisions(rp):
    """The device decides 'identical views' (empty response, convergence, the
    checksum dedupe's leaders) by 64-bit view fingerprints where the reference
    compares farmhash checksums (lib/dissemination.js:102-117, tick-cluster's
    convergence).  Views one minimal edit apart from a common base -- two
    incarnations swapped, suspect vs alive at the same incarnation, faulty vs
    leave vs absent, incarnation + 1 -- must give the decisions the oracle
    takes by real checksums, round for round, and checksum classes equal to
    view classes."""
    n, seed = 64, 11
    base_inc = 1434401518824 + np.arange(n, dtype=np.int64)
    st = np.ones((n, n), dtype=np.int32)
    inc = np.tile(base_inc, (n, 1))
    inc[1, 10], inc[1, 11] = base_inc[11], base_inc[10]  # two incarnations swapped
    inc[2, 11], inc[2, 10] = base_inc[11], base_inc[10]  # the same cells written in the other order: no edit
    st[3, 12] = 2                                          # suspect at the same incarnation
    st[4, 13] = 3                                          # faulty ...
    st[5, 13] = 4                                          # ... vs leave ...
    st[6, 13] = 0                                          # ... vs absent
    inc[7, 14] += 1                                        # incarnation + 1
    inc[8, 14] += 1                                        # the same edit on another node: equal views
    st[9, 15], st[9, 16] = 2, 2                            # two suspects ...
    st[10, 15], inc[10, 16] = 2, base_inc[16] + 1          # ... vs one suspect and a bumped alive
    g = rp.Sim(n, seed, churn_k=0, views=(st, inc))
    c = oracle.Sim(n, seed, churn_k=0, views=(st, inc))

    def classes(keys):
        first = {}
        return [first.setdefault(k, i) for i, k in enumerate(keys)]

    views0 = []
    for v in range(n):
        s, i = g.view(v)
        views0.append((s.tobytes(), i.tobytes()))
    gc0 = g.checksums().tolist()
    assert classes(gc0) == classes(views0)
    assert len(set(classes(views0))) == 9  # 0, 2, 11.. | 1 | 3 | 4 | 5 | 6 | 7, 8 | 9 | 10
    assert gc0 == [x if x is not None else gc0[i] for i, x in enumerate(c.checksums())]
    for rnd in range(12):
        go, co = g.round(churn=False), c.round(churn=False)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert go[key] == co[key], (rnd, key)
        gc = g.checksums().tolist()
        assert gc == [x if x is not None else gc[i] for i, x in enumerate(c.checksums())], rnd
