"""Wire-format bridge on the GPU (rp_sim_ping_body / rp_sim_handle_ping /
rp_sim_update + ringpop_amd/wire.py): the reference's own JSON ping bodies
and responses (tests/golden/wire_bridge.json), on one and two shards, and
random bridge traffic against the oracle."""
import json

import numpy as np
import pytest

import oracle
from wire_cases import replay, run_rounds, sim_args, strip_ids

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rp(gpu_lib):
    import ringpop_amd
    return ringpop_amd


@pytest.mark.parametrize("idx,shards", [(0, 1), (1, 1), (0, 2), (1, 4)])
def test_bridge_rows_against_reference(rp, golden, idx, shards):
    case = golden("wire_bridge.json")["cases"][idx]
    cfg = case["config"]
    S = rp.Sim(cfg["n"], cfg["seed"], shards=shards, **sim_args(cfg))
    run_rounds(S, cfg)
    assert S.addresses() == case["addresses"]
    replay(S, case, case["addresses"])


@pytest.mark.parametrize("idx", [0, 1])
def test_bridge_json_against_reference(rp, golden, idx):
    """SimNodeWire end to end: JSON strings in, JSON strings out."""
    from ringpop_amd.wire import SimNodeWire
    case = golden("wire_bridge.json")["cases"][idx]
    cfg = case["config"]
    S = rp.Sim(cfg["n"], cfg["seed"], **sim_args(cfg))
    run_rounds(S, cfg)
    for k, op in enumerate(case["bridge"]):
        o = op["op"]
        if o["op"] == "ping":
            body = SimNodeWire(S, o["from"]).ping_body()
            b = json.loads(body)
            assert b == {**op["body"], "changes": strip_ids(op["body"]["changes"])}, k
            assert list(b) == ["checksum", "changes", "source", "sourceIncarnationNumber"]
        else:
            body = json.dumps(o["body"])
        resp = SimNodeWire(S, o["to"]).handle_ping(body)
        assert json.loads(resp) == {"changes": strip_ids(op["response"]["changes"])}, k
        if o["op"] == "ping":
            assert SimNodeWire(S, o["from"]).on_ping_response(json.dumps(op["response"])) == op["applied"], k
    with pytest.raises(ValueError):
        SimNodeWire(S, 0).handle_ping('{"source": "x", "changes": []}')  # no checksum: rejected like the endpoint


def test_bridge_random_traffic_against_oracle(rp):
    """Random pings between nodes and injected bodies after a run with
    churn, a fail-stop and a partition: every list, count and dump equals the
    oracle's, and the rounds that follow stay identical."""
    n, seed = 128, 31
    fail = {2: [5, 77]}
    part = {"start": 4, "end": 9, "split": 50}
    g = rp.Sim(n, seed, churn_k=2, failures=fail, partition=part)
    c = oracle.Sim(n, seed, churn_k=2, failures=fail, partition=part)
    for r in range(14):
        g.round(churn=r < 10)
        c.round(churn=r < 10)
    rng = np.random.default_rng(7)
    live = [v for v in range(n) if v not in (5, 77)]
    for k in range(40):
        a, b = (int(x) for x in rng.choice(live, size=2, replace=False))
        if k % 4 == 3:  # a foreign body: random suspect / faulty / alive claims
            st_a, inc_a = c.view(a)
            addrs = rng.choice(n, size=5, replace=False)
            rows = np.array([[x, int(rng.integers(1, 4)), int(inc_a[x]) + int(rng.integers(0, 2)), a, int(inc_a[a])]
                             for x in addrs], dtype=np.int64)
            src, sinc, cs = a, int(inc_a[a]), int(rng.integers(1, 2**32))
        else:
            rows, cs, sinc = c.ping_body(a)
            grows, gcs, gsinc = g.ping_body(a)
            assert grows.tolist() == rows.tolist() and gcs == cs and gsinc == sinc, k
            src = a
        ro, ao, fo = c.handle_ping(b, src, sinc, cs, rows)
        rg, ag, fg = g.handle_ping(b, src, sinc, cs, rows)
        assert rg.tolist() == ro.tolist() and ag == ao and fg == fo, k
        if k % 4 != 3:
            assert g.update(a, ro) == c.update(a, ro), k
        for v in (a, b):
            assert g.changes(v).tolist() == c.changes(v).tolist(), (k, v)
            assert np.array_equal(g.view(v)[1], c.view(v)[1]), (k, v)
            assert g.checksum(v) == c.checksum(v), (k, v)
    for r in range(10):
        x, y = g.round(churn=True), c.round(churn=True)
        for key in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged"):
            assert x[key] == y[key], (r, key)
        cs_g = g.checksums().tolist()
        assert [u if w is not None else None for u, w in zip(cs_g, c.checksums())] == c.checksums(), r
