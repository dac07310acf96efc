"""GPU parity of one ringpop instance's Membership / Dissemination on the
device (rp_node_*, ringpop_amd/node.py) against fixtures the reference's own
code produced (oracle/harness/gen_golden.js): the rules truth table, config 1
(benchmarks/large-membership.json into a ready instance: unknown members
spliced at getJoinPosition) and seeded operation sequences through the whole
drop-in surface."""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def rp(gpu_lib):
    import ringpop_amd
    return ringpop_amd


class Instance:
    """A ringpop instance's hot-path objects on the device, wired like
    RingPop wires them: the update / set listeners
    (lib/membership-update-listener.js:24-75, lib/membership-set-listener.js:
    24-48) feed HashRing.addRemoveServers and Dissemination.recordChange, and
    'ringChanged' adjusts maxPiggybackCount (lib/dissemination.js:121-123)."""

    def __init__(self, rp, whoami, seed, now=1500000000000):
        self.now = now
        self.node = rp.Node(whoami, rng_state=seed)
        self.ring = rp.HashRing()
        self.membership = rp.Membership(self.node, ready=True, now=lambda: self.now, on_updated=self._updated)
        self.dissemination = rp.Dissemination(self.node, self.membership)

    def _updated(self, updates):
        add, rm = [], []
        for u in updates:
            if u["status"] == "alive":
                add.append(u["address"])
            elif u["status"] in ("faulty", "leave"):
                rm.append(u["address"])
            self.dissemination.recordChange(u)
        if add or rm:
            if self.ring.addRemoveServers(add, rm):
                self.dissemination.adjustMaxPiggybackCount(self.ring.getServerCount())

    def close(self):
        self.node.close()
        self.ring.close()


def test_rules_truth_table_through_device_merge(rp, golden):
    """Every (current, change) status pair x incarnation relation x self/other
    (lib/membership-update-rules.js:25-59, local override :244-254)."""
    g = golden("rules_truth_table.json")
    for c in g["cases"]:
        inst = Instance(rp, "127.0.0.1:3000", 1, now=g["now"])
        m = inst.membership
        m.makeAlive("127.0.0.1:3000", 1000)
        target = "127.0.0.1:3000" if c["self"] else "127.0.0.1:3001"
        if not c["self"]:
            m.makeAlive(target, 1000)
        m.force(target, c["current"], 1000)
        applied = m.update([{"address": target, "status": c["change"], "incarnationNumber": 1000 + c["rel"],
                             "source": "127.0.0.1:3009", "sourceIncarnationNumber": 7}])
        got = m.findMemberByAddress(target)
        assert (len(applied), got["status"], got["incarnationNumber"]) == (c["applied"], c["status"], c["inc"]), c
        inst.close()


@pytest.mark.parametrize("size", [100, 1000, 1332])
def test_config1_large_membership_update(rp, golden, size):
    """Config 1: update(large-membership.json[:size]) into a ready instance
    (benchmarks/large-membership-update.js:37-47 with isReady set): applied
    count, member order (getJoinPosition splices), checksum string and
    checksum (compute-checksum.js:46-62), ring, dissemination key order."""
    g = golden("config1_large_membership.json")
    want = g["results"][str(size)]
    recs = golden("large_membership_input.json")[:size]
    inst = Instance(rp, "127.0.0.1:3000", g["seed_base"] + size)
    applied = inst.membership.update([dict(r) for r in recs])
    assert len(applied) == want["applied"]
    assert [x["address"] for x in inst.membership.members] == want["members_order"]
    s = inst.membership.generateChecksumString().encode()
    assert len(s) == want["checksum_string_len"]
    assert hashlib.sha256(s).hexdigest() == want["checksum_string_sha"]
    assert inst.membership.checksum == want["checksum"]
    assert inst.ring.getServerCount() == want["ring_servers"] and inst.ring.checksum == want["ring_checksum"]
    assert inst.dissemination.maxPiggybackCount == want["max_piggyback"]
    assert list(inst.dissemination.changes) == want["changes"]
    inst.close()


def _state(inst):
    d = inst.dissemination
    return {
        "checksum": inst.membership.checksum,
        "members": [[m["address"], m["status"], m["incarnationNumber"]] for m in inst.membership.members],
        "changes": [[a, c["status"], c["incarnationNumber"], c.get("source"), c.get("sourceIncarnationNumber"),
                     c.get("piggybackCount")] for a, c in d.changes.items()],
        "maxPiggybackCount": d.maxPiggybackCount,
        "ringServers": inst.ring.getServerCount(), "ringChecksum": inst.ring.checksum,
    }


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_node_op_sequences_against_reference(rp, golden, idx):
    """150 seeded operations through Membership / Dissemination / HashRing:
    results and the whole instance state after every op equal the
    reference's."""
    case = golden("node_ops.json.gz")["cases"][idx]
    inst = Instance(rp, case["self"], 1000 + case["seed"])
    m, d = inst.membership, inst.dissemination
    for k, op in enumerate(case["ops"]):
        inst.now = 1500000000000 + max(k - 1, 0)
        kind = op["op"]
        res = None
        if kind == "update":
            res = m.update([dict(c) for c in op["changes"]])
        elif kind in ("makeAlive", "makeSuspect", "makeFaulty"):
            res = getattr(m, kind)(op["address"], op["incarnationNumber"])
        elif kind == "issueAsSender":
            res = d.issueAsSender()
        elif kind == "issueAsReceiver":
            res = d.issueAsReceiver(op["sender"], op["senderIncarnationNumber"], op["senderChecksum"])
        elif kind == "fullSync":
            res = d.fullSync()
        elif kind == "shuffle":
            m.shuffle()
        elif kind == "clearChanges":
            d.clearChanges()
        if "result" in op:
            keys = ("source", "sourceIncarnationNumber", "address", "status", "incarnationNumber")
            got = [{kk: c[kk] for kk in keys if c.get(kk) is not None} for c in res]
            assert got == op["result"], (k, kind)
        assert _state(inst) == op["state"], (k, kind)
    inst.close()


def test_set_merges_changesets(rp):
    """Membership.set (lib/membership.js:162-206) with
    mergeMembershipChangesets (lib/membership-changeset-merge.js:22-51; cases
    of test/membership-changeset-merge-test.js:26-63): max incarnation per
    address, the first of equals, first-appearance order, self skipped,
    members pushed at the end."""
    node = rp.Node("127.0.0.1:3000", rng_state=5)
    sets = []
    m = rp.Membership(node, ready=False, on_set=sets.append)
    m.makeAlive("127.0.0.1:3000", 1)  # isLocal: applied before ready
    m.update([{"address": "127.0.0.1:3001", "status": "alive", "incarnationNumber": 1},
              {"address": "127.0.0.1:3002", "status": "suspect", "incarnationNumber": 5, "source": "a"}])
    m.update([{"address": "127.0.0.1:3002", "status": "alive", "incarnationNumber": 7},
              {"address": "127.0.0.1:3000", "status": "faulty", "incarnationNumber": 99},
              {"address": "127.0.0.1:3003", "status": "faulty", "incarnationNumber": 3},
              {"address": "127.0.0.1:3001", "status": "suspect", "incarnationNumber": 1}])
    assert m.getMemberCount() == 1 and len(m.stashedUpdates) == 2
    m.set()
    assert m.stashedUpdates is None
    assert [u["address"] for u in sets[0]] == ["127.0.0.1:3001", "127.0.0.1:3002", "127.0.0.1:3003"]
    assert [(u["status"], u["incarnationNumber"]) for u in sets[0]] == [("alive", 1), ("alive", 7), ("faulty", 3)]
    assert [x["address"] for x in m.members] == ["127.0.0.1:3000", "127.0.0.1:3001", "127.0.0.1:3002",
                                                 "127.0.0.1:3003"]
    assert m.checksum == m.computeChecksum()
    node.close()


def test_update_large_batch_of_unknown_members(rp):
    """A full sync's worth of unknown members (65,536) spliced at once: the
    member order equals the sequential splice definition."""
    n = 65536
    node = rp.Node("10.0.0.0:3000", rng_state=77)
    m = rp.Membership(node, ready=True)
    addrs = [f"10.{i >> 16 & 255}.{i >> 8 & 255}.{i & 255}:{3000 + i % 7}" for i in range(n)]
    changes = [{"address": a, "status": "alive", "incarnationNumber": 1434401518824 + i} for i, a in enumerate(addrs)]
    applied = m.update(changes)
    assert len(applied) == n
    # getJoinPosition with the instance's stream: draw j = floor(random_j * j)
    import oracle  # noqa: F401  (checker: the splitmix stream restated in numpy)
    G = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        s = np.uint64(77) + (np.arange(n, dtype=np.uint64) + np.uint64(1)) * G
        z = (s ^ (s >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    x = (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    pos = np.floor(x * np.arange(n)).astype(np.int64)
    order = []
    for j in range(n):
        order.insert(int(pos[j]), j)
    assert [x["address"] for x in m.members] == [addrs[j] for j in order]
    assert m.checksum == m.computeChecksum()
    node.close()


def test_record_many_changes_to_few_addresses(rp):
    """Dissemination.recordChange upserts by address (lib/dissemination.js:
    125-127): an overwritten key keeps its place and the table holds one key
    per address, however many changes arrive between two issues.  Recording
    3 x 1,000 changes of 3 addresses in one batch (the JS host queues every
    recordChange until the next issue), then 2,500 more one call at a time,
    must not outgrow the device log (the room reserved used to be
    the raw batch length) and must issue exactly the reference's list."""
    node = rp.Node("10.0.0.1:3000", rng_state=3)
    d = rp.Dissemination(node)
    d.maxPiggybackCount = 5
    addrs = ["10.0.0.2:3000", "10.0.0.3:3000", "10.0.0.4:3000"]
    want = {}
    batch = []
    for i in range(3000):
        c = {"address": addrs[i % 3] if i % 7 else addrs[(i // 7) % 3], "status": ("alive", "suspect", "faulty")[i % 3],
             "incarnationNumber": 1000 + i, "source": "10.0.0.9:3000", "sourceIncarnationNumber": 7}
        batch.append(c)
        want[c["address"]] = c  # JS object: overwrite keeps the key's insertion position
    d.recordChanges(batch)
    for i in range(2500):
        c = {"address": addrs[(i * 5) % 3], "status": "alive", "incarnationNumber": 5000 + i}
        d.recordChange(c)
        want[c["address"]] = c
    got = d.issueAsSender()
    assert [g["address"] for g in got] == list(want)
    for g in got:
        w = want[g["address"]]
        assert (g["status"], g["incarnationNumber"]) == (w["status"], w["incarnationNumber"])
        assert g.get("source") == w.get("source")
    assert len(d.changes) == 3
    node.close()
