"""Replays the wire-bridge fixture (tests/golden/wire_bridge.json, made by
oracle/harness/gen_golden.js from the reference's own ping path) on a
simulation object -- the oracle (CPU tests) or the device (GPU tests) -- and
checks every JSON body, response, applied count and node dump.  The
reference's change ids (uuids) are not modelled and are dropped."""
import numpy as np

from ringpop_amd import wire


def strip_ids(changes):
    return [{k: v for k, v in c.items() if k != "id"} for c in changes]


def run_rounds(S, cfg):
    for r in range(cfg["maxRounds"]):
        S.round(churn=r < cfg["churnRounds"])


def check_dump(S, v, d):
    st, inc = S.view(v)
    for a, e in enumerate(d["view"]):
        assert (int(st[a]), int(inc[a])) == ((0, 0) if e is None else tuple(e)), (v, a)
    assert S.members(v).tolist() == d["members"], v
    assert S.changes(v).tolist() == d["changes"], v
    info = S.info(v)
    assert info["max_pb"] == d["maxPiggyback"] and info["ring_servers"] == d["ringServers"], v
    assert info["ring_checksum"] == d["ringChecksum"], v
    assert S.checksum(v) == d["checksum"], v


def replay(S, case, addresses):
    """Run the case's bridge ops through S's row-level API + the product codec."""
    index = {a: i for i, a in enumerate(addresses)}
    enc = lambda rows: [wire.change_json(r, addresses) for r in rows]  # noqa: E731
    for k, op in enumerate(case["bridge"]):
        o = op["op"]
        if o["op"] == "ping":
            rows, cs, inc = S.ping_body(o["from"])
            body = {"checksum": cs, "changes": enc(rows), "source": addresses[o["from"]],
                    "sourceIncarnationNumber": inc}
            assert body == {**op["body"], "changes": strip_ids(op["body"]["changes"])}, k
        else:
            body = o["body"]
        resp, applied_to, fs = S.handle_ping(o["to"], index.get(body["source"], -1),
                                             int(body.get("sourceIncarnationNumber") or 0), int(body["checksum"]),
                                             wire.changes_rows(body["changes"], index))
        assert enc(resp) == strip_ids(op["response"]["changes"]), k
        if o["op"] == "ping":
            applied = S.update(o["from"], wire.changes_rows(op["response"]["changes"], index))
            assert applied == op["applied"], k
            check_dump(S, o["from"], op["fromDump"])
        check_dump(S, o["to"], op["toDump"])


def sim_args(cfg):
    fail = {int(k): v for k, v in cfg.get("failures", {}).items()}
    return dict(churn_k=cfg.get("churnK"), failures=fail)


def gpu_checksum(S, v):
    return int(S.checksums()[v])


__all__ = ["replay", "run_rounds", "sim_args", "strip_ids", "np"]
