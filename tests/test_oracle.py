"""CPU tests: the oracle (C restatement) against the reference's golden vectors.

The fixtures in tests/golden/ were produced by oracle/harness/gen_golden.js,
which runs the UNMODIFIED reference JavaScript from /root/reference.
"""
import numpy as np
import pytest

import oracle


def test_farmhash_known_answers():
    # upstream farmhash test table, first entries (len 0): Hash32 and
    # Hash32WithSeed(CreateSeed(0,-1)) -- pins c1/c2, Mur, fmix, len<=4 branch
    assert oracle.farmhash32(b"") == 0xDC56D17A == 3696677242
    L = oracle.lib()
    assert L.oracle_farmhash32_seed(b"", 0, L.oracle_farmhash_test_seed(0, -1)) == 4223616069


def test_farmhash_js_transcription_matches_c(golden):
    g = golden("farmhash_vectors.json")
    got = oracle.farmhash32_batch(g["strings"])
    assert got.tolist() == g["hash32"]


def test_max_piggyback_table(golden):
    for count, want in golden("max_piggyback.json")["table"]:
        assert oracle.max_piggyback(count) == want, count


def test_rules_truth_table(golden):
    g = golden("rules_truth_table.json")
    code = {"alive": 1, "suspect": 2, "faulty": 3, "leave": 4}
    for c in g["cases"]:
        st = np.array([1, 1], dtype=np.uint8)
        inc = np.array([1000, 1000], dtype=np.uint64)
        tgt = 0 if c["self"] else 1
        st[tgt] = code[c["current"]]
        addr = np.array([tgt], dtype=np.int32)
        cst = np.array([code[c["change"]]], dtype=np.uint8)
        cinc = np.array([1000 + c["rel"]], dtype=np.uint64)
        ap = np.zeros(1, dtype=np.uint8)
        n = oracle.lib().orc_view_update(0, g["now"], oracle._ptr(st), oracle._ptr(inc), 1, oracle._ptr(addr),
                                         oracle._ptr(cst), oracle._ptr(cinc), oracle._ptr(ap))
        assert n == c["applied"], c
        assert st[tgt] == code[c["status"]] and inc[tgt] == c["inc"], c


def test_config1_checksums(golden):
    """Config 1 (benchmarks/large-membership.json): checksum strings of the ready view."""
    import hashlib
    import json
    import os
    g = golden("config1_large_membership.json")
    path = os.path.join(os.path.dirname(__file__), "golden", "large_membership_input.json")
    data = json.load(open(path))
    code = {"alive": 1, "suspect": 2, "faulty": 3, "leave": 4}
    for size, want in g["results"].items():
        recs = data[: int(size)]
        addrs = sorted({r["address"] for r in recs})
        idx = {a: i for i, a in enumerate(addrs)}
        st = np.zeros(len(addrs), dtype=np.uint8)
        inc = np.zeros(len(addrs), dtype=np.uint64)
        for r in recs:  # update() into an empty view: every record is new (first wins)
            i = idx[r["address"]]
            if st[i] == 0:
                st[i] = code[r["status"]]
                inc[i] = r["incarnationNumber"]
        blob = "".join(addrs).encode()
        off = np.zeros(len(addrs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(a) for a in addrs])
        b = np.frombuffer(blob, dtype=np.uint8)
        buf = np.zeros(len(blob) + 40 * len(addrs), dtype=np.uint8)
        L = oracle.lib().orc_checksum_string(oracle._ptr(b), oracle._ptr(off), len(addrs), oracle._ptr(st),
                                             oracle._ptr(inc), oracle._ptr(buf), len(buf))
        s = bytes(buf[:L])
        assert L == want["checksum_string_len"]
        assert hashlib.sha256(s).hexdigest() == want["checksum_string_sha"]
        assert oracle.farmhash32(s) == want["checksum"]


def views_of(cfg):
    """cfg["views"][i][j] = [status, incarnation] -> (status, inc) arrays, or None"""
    if "views" not in cfg:
        return None
    v = np.array(cfg["views"], dtype=np.int64)
    return v[:, :, 0], v[:, :, 1]


def _run_case(case):
    cfg = case["config"]
    fail = {int(k): v for k, v in cfg.get("failures", {}).items()}
    S = oracle.Sim(cfg["n"], cfg["seed"], churn_k=cfg.get("churnK"), failures=fail,
                   partition=cfg.get("partition"), storm=cfg.get("storm"), addresses=cfg.get("addresses"),
                   views=views_of(cfg), joins=[tuple(e) for e in cfg.get("joins", [])] or None)
    for r, jr in enumerate(case["rounds"]):
        o = S.round(churn=r < cfg["churnRounds"])
        assert o["churned"] == jr["churned"], r
        for k, jk in (("evaluated", "evaluated"), ("applied", "applied"), ("full_syncs", "fullSyncs"),
                      ("messages", "messages"), ("waves", "waves")):
            assert o[k] == jr[jk], (r, k)
        assert S.checksums() == jr["checksums"], r
        assert bool(o["converged"]) == jr["converged"], r
    return S


def _check_final(S, final):
    for v, f in enumerate(final):
        st, inc = S.view(v)
        for a, e in enumerate(f["view"]):
            assert (st[a], inc[a]) == ((0, 0) if e is None else tuple(e)), (v, a)
        assert S.members(v).tolist() == f["members"], v
        assert S.changes(v).tolist() == f["changes"], v
        info = S.info(v)
        assert info["max_pb"] == f["maxPiggyback"] and info["ring_servers"] == f["ringServers"]
        if f["ringChecksum"] is not None:  # (an empty ring never computed one: a node that never joined)
            assert info["ring_checksum"] == f["ringChecksum"]
        assert info["iter_index"] == f["iterIndex"] and info["iter_round"] == f["iterRound"]
        assert (info["rng"] & (2**64 - 1)) == int(f["rng"])
        assert sorted(S.timers(v).tolist()) == sorted(f["timers"])


@pytest.mark.parametrize("idx", range(5))
def test_sim_small_against_reference(golden, idx):
    case = golden("sim_small.json.gz")["cases"][idx]
    S = _run_case(case)
    _check_final(S, case["final"])


@pytest.mark.parametrize("idx", range(2))
def test_sim_medium_against_reference(golden, idx):
    case = golden("sim_medium.json.gz")["cases"][idx]
    S = _run_case(case)
    assert [S.checksum(v) for v in range(S.n)] == case["final_checksums"]


@pytest.mark.parametrize("idx", range(3))
def test_sim_storm_against_reference(golden, idx):
    """Config 5's false-suspicion storm (makeSuspect + refutes) against the reference."""
    case = golden("sim_storm.json.gz")["cases"][idx]
    S = _run_case(case)
    if "final" in case:
        _check_final(S, case["final"])
    else:
        assert [S.checksum(v) for v in range(S.n)] == case["final_checksums"]


@pytest.mark.parametrize("idx", range(4))
def test_sim_views_against_reference(golden, idx):
    """Arbitrary clusters: loaded addresses (4-32 bytes) and per-node bootstrap
    views with suspects (timers due at round 0), faulty and leave members."""
    case = golden("sim_views.json.gz")["cases"][idx]
    S = _run_case(case)
    if "final" in case:
        _check_final(S, case["final"])
    else:
        assert [S.checksum(v) for v in range(S.n)] == case["final_checksums"]


@pytest.mark.parametrize("idx", range(4))
def test_sim_join_against_reference(golden, idx):
    """The join path: nodes outside the cluster join through seeds
    (handleJoin, mergeJoinResponses, set()) and gossip splices them in."""
    case = golden("sim_join.json.gz")["cases"][idx]
    S = _run_case(case)
    if "final" in case:
        _check_final(S, case["final"])
    else:
        assert [S.checksum(v) for v in range(S.n)] == case["final_checksums"]


def test_sim_config2_n1024_against_reference(golden):
    case = golden("sim_config2_n1024.json.gz")["cases"][0]
    S = _run_case(case)
    assert case["convergedAt"] == len(case["rounds"]) - 1


def test_numpy_ring_restatement_matches_c_oracle(golden):
    """oracle.ring_points_add_only / ring_lookup_points (used at config-3 scale,
    where the C oracle's array inserts are too slow) against the C oracle ring
    and the reference's ring fixture."""
    import numpy as np
    g = golden("ring_farmhash.json")
    h, o = oracle.ring_points_add_only(g["servers"])
    L = oracle.lib()
    r = L.orc_ring_new(100)
    bs = [s.encode() for s in g["servers"]]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
    L.orc_ring_add_remove(r, oracle._ptr(blob), oracle._ptr(off), len(bs), None, None, None, 0, None)
    H = np.zeros(len(bs) * 100, dtype=np.uint32)
    O = np.zeros(len(bs) * 100, dtype=np.int32)
    k = L.orc_ring_points(r, oracle._ptr(H), oracle._ptr(O))
    L.orc_ring_free(r)
    assert np.array_equal(H[:k], h) and np.array_equal(O[:k], o)
    owners = oracle.ring_lookup_points(h, o, oracle.farmhash32_batch(g["keys"]))
    assert [g["servers"][i] for i in owners] == g["owners"]
    # config-3 key strings: decimal splitmix64 values (rp_ring_make_keys_device)
    assert oracle.lookup_keys(5, [0, 1]) == ["7134611160154358618", "13877614986023876344"]


def test_group_by_owner_restatements_agree(golden):
    """handleOrProxyAll grouping: the per-key restatement and the argsort one agree,
    and regrouping the reference fixture's owners gives first-appearance order."""
    g = golden("ring_farmhash.json")
    names = {s: i for i, s in enumerate(g["servers"])}
    owners = np.array([names[o] for o in g["owners"]], dtype=np.int32)
    a, b = oracle.group_by_owner(owners), oracle.group_by_owner_np(owners)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    seen = []
    for o in owners.tolist():
        if o not in seen:
            seen.append(o)
    assert a[0].tolist() == seen
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 5000):
        o = rng.integers(-1, 50, size=n)
        a, b = oracle.group_by_owner(o), oracle.group_by_owner_np(o)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
