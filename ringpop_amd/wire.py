"""Wire-format bridge: the reference's JSON ping bodies for simulated nodes.

A real ringpop process and the device simulation can exchange gossip through
the same bodies ringpop puts on the wire:

* ping request (lib/swim/ping-sender.js:70-76):
  ``{"checksum", "changes", "source", "sourceIncarnationNumber"}``
* ping response (server/ping-handler.js:36-39, server/index.js:175-192):
  ``{"changes"}``

Changes are the issueAs copy (lib/dissemination.js:170-177): ``source``,
``sourceIncarnationNumber``, ``address``, ``status``, ``incarnationNumber`` in
that order, undefined fields omitted as JSON.stringify omits them.  The
reference's per-change ``id`` (a uuid minted by makeUpdate, carried along but
read by nothing on this path) is not modelled: the device emits none and
ignores incoming ones.

``SimNodeWire`` mirrors the three call sites: ``ping_body`` (PingSender.send),
``handle_ping`` (RingPopTChannel.protocolPing -> handlePing) and
``on_ping_response`` (PingSender.onPing).  All run on the GPU through the C ABI
(rp_sim_ping_body / rp_sim_handle_ping / rp_sim_update).
"""
import json

import numpy as np

STATUS = {1: "alive", 2: "suspect", 3: "faulty", 4: "leave"}
STATUS_CODE = {v: k for k, v in STATUS.items()}


def _dumps(obj):
    return json.dumps(obj, separators=(",", ":"))


def _truthy(x):
    """JavaScript truthiness of a parsed JSON value ([] and {} are truthy)."""
    return not (x is None or x is False or x == 0 or x == "")


def change_json(row, addresses):
    """One change row -> the issueAs copy (undefined fields omitted)."""
    addr, status, inc, src, src_inc = (int(x) for x in row)
    c = {}
    if src >= 0:
        c["source"] = addresses[src]
    if src_inc:
        c["sourceIncarnationNumber"] = src_inc
    c["address"] = addresses[addr]
    c["status"] = STATUS[status]
    c["incarnationNumber"] = inc
    return c


def changes_rows(changes, index):
    """JSON changes -> rows; `index` maps address strings to member ids."""
    rows = np.zeros((len(changes), 5), dtype=np.int64)
    for i, c in enumerate(changes):
        rows[i, 0] = index[c["address"]]
        rows[i, 1] = STATUS_CODE[c["status"]]
        rows[i, 2] = int(c["incarnationNumber"])
        src = c.get("source")
        rows[i, 3] = index[src] if src else -1
        rows[i, 4] = int(c.get("sourceIncarnationNumber") or 0)
    return rows


class SimNodeWire:
    """The ping wire surface of node `v` of a ringpop_amd.Sim."""

    def __init__(self, sim, v):
        self.sim, self.v = sim, v
        self.addresses = sim.addresses()
        self.index = {a: i for i, a in enumerate(self.addresses)}

    def ping_body(self):
        """PingSender.send's body (lib/swim/ping-sender.js:70-76)."""
        rows, checksum, inc = self.sim.ping_body(self.v)
        return _dumps({"checksum": checksum, "changes": [change_json(r, self.addresses) for r in rows],
                       "source": self.addresses[self.v], "sourceIncarnationNumber": inc})

    def handle_ping(self, body):
        """/protocol/ping (server/index.js:175-192 -> server/ping-handler.js:22-40):
        the response body, or ValueError as the endpoint rejects bad bodies."""
        try:
            b = json.loads(body)
        except ValueError:
            b = None
        if not isinstance(b, dict) or not _truthy(b.get("source")) or not _truthy(b.get("changes")) or \
                not _truthy(b.get("checksum")):
            raise ValueError("need req body with source, changes, and checksum")
        src = self.index.get(b["source"], -1)
        rows, _, _ = self.sim.handle_ping(self.v, src, int(b.get("sourceIncarnationNumber") or 0), int(b["checksum"]),
                                          changes_rows(b["changes"], self.index))
        return _dumps({"changes": [change_json(r, self.addresses) for r in rows]})

    def on_ping_response(self, response):
        """PingSender.onPing (lib/swim/ping-sender.js:30-44): Membership.update with
        the response's changes; returns the number applied (None: bad body)."""
        try:
            b = json.loads(response)
        except ValueError:
            return None
        if not isinstance(b, dict) or not _truthy(b.get("changes")):
            return None
        return self.sim.update(self.v, changes_rows(b["changes"], self.index))
