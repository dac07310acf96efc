"""Wire-format bridge, CPU side: the oracle's node-level ping path and the
product's JSON codec (ringpop_amd/wire.py) against the reference's own
bodies (tests/golden/wire_bridge.json)."""
import json

import pytest

import oracle
from ringpop_amd import wire
from wire_cases import replay, run_rounds, sim_args


@pytest.mark.parametrize("idx", [0, 1])
def test_oracle_bridge_against_reference(golden, idx):
    case = golden("wire_bridge.json")["cases"][idx]
    cfg = case["config"]
    S = oracle.Sim(cfg["n"], cfg["seed"], **sim_args(cfg))
    run_rounds(S, cfg)
    assert [S.address(i) for i in range(cfg["n"])] == case["addresses"]
    replay(S, case, case["addresses"])


def test_codec_round_trip(golden):
    """changes JSON -> rows -> JSON is the identity on the reference's own
    bodies (ids aside), key order included (injected bodies are hand-written)."""
    case = golden("wire_bridge.json")["cases"][0]
    index = {a: i for i, a in enumerate(case["addresses"])}
    for op in case["bridge"]:
        lists = [op["response"]["changes"]] + ([op["body"]["changes"]] if op["op"]["op"] == "ping" else [])
        for ch in lists:
            rows = wire.changes_rows(ch, index)
            back = [wire.change_json(r, case["addresses"]) for r in rows]
            want = [{k: v for k, v in c.items() if k != "id"} for c in ch]
            assert json.dumps(back) == json.dumps(want)


def test_codec_js_truthiness():
    assert wire._truthy([]) and wire._truthy({}) and wire._truthy("x")
    assert not any(wire._truthy(x) for x in (None, False, 0, ""))
