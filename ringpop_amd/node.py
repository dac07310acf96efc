"""One ringpop instance's Membership and Dissemination on the device (rp_node_*).

Python mirror of the reference's classes (lib/membership.js:31-354,
lib/dissemination.js:27-184) over the C ABI, with the reference's method
names, argument meanings and results; changes are dicts with the reference's
field names.  State lives on the GPU: the member table and order, the
insertion-ordered change table with piggyback counts, and the instance's
Math.random stream (getJoinPosition / shuffle / sample).
There is no CPU fallback: without the library or a GPU every call raises.
"""
import ctypes

import numpy as np

from ._lib import check, lib, ptr

STATUS_CODE = {"alive": 1, "suspect": 2, "faulty": 3, "leave": 4}
STATUS_NAME = {v: k for k, v in STATUS_CODE.items()}


class MemberChange(ctypes.Structure):
    _fields_ = [("address", ctypes.c_int64), ("incarnation", ctypes.c_int64), ("source", ctypes.c_int64),
                ("source_incarnation", ctypes.c_int64), ("status", ctypes.c_int32), ("piggyback", ctypes.c_int32),
                ("reserved", ctypes.c_int64)]


ROW = np.dtype([("address", "<i8"), ("incarnation", "<i8"), ("source", "<i8"), ("source_incarnation", "<i8"),
                ("status", "<i4"), ("piggyback", "<i4"), ("reserved", "<i8")])
assert ROW.itemsize == ctypes.sizeof(MemberChange) == 48


def _inc(x):
    if x is None:
        return -1
    if not isinstance(x, (int, np.integer)) or x < 0 or x >= 2 ** 53:
        raise ValueError(f"incarnation numbers must be integers in [0, 2^53): {x!r}")
    return int(x)


class Node:
    """The device state of one ringpop instance (rp_node)."""

    def __init__(self, whoami, rng_state=0):
        b = whoami.encode()
        self._h = ctypes.c_void_p()
        check(lib().rp_node_create(ctypes.c_char_p(b), len(b), ctypes.c_uint64(rng_state & (2**64 - 1)),
                                   ctypes.byref(self._h)))
        self.names = [whoami]
        self.ids = {whoami: 0}

    def close(self):
        if self._h:
            lib().rp_node_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def intern(self, addresses):
        """ids of `addresses`, new ones assigned in first-seen order (mirrors rp_node_intern)."""
        new = [a for a in dict.fromkeys(addresses) if a not in self.ids]
        if new:
            bs = [a.encode() for a in new]
            off = np.zeros(len(bs) + 1, dtype=np.uint64)
            off[1:] = np.cumsum([len(x) for x in bs])
            blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
            out = np.zeros(len(bs), dtype=np.uint32)
            check(lib().rp_node_intern(self._h, ptr(blob), ptr(off), len(bs), ptr(out)))
            for a, i in zip(new, out.tolist()):
                assert i == len(self.names)
                self.ids[a] = i
                self.names.append(a)
        return [self.ids[a] for a in addresses]

    @property
    def rng_state(self):
        v = ctypes.c_uint64(0)
        check(lib().rp_node_rng(self._h, ctypes.byref(v), None))
        return v.value

    @rng_state.setter
    def rng_state(self, s):
        v = ctypes.c_uint64(s & (2**64 - 1))
        check(lib().rp_node_rng(self._h, None, ctypes.byref(v)))

    # -- rows <-> change dicts
    def rows(self, changes):
        r = np.zeros(len(changes), dtype=ROW)
        addrs = [c.get("address") for c in changes]
        ids = self.intern([a for a in addrs if a is not None] + [c["source"] for c in changes
                                                                   if c.get("source") is not None])
        it = iter(ids)
        for k, c in enumerate(changes):
            r[k]["address"] = next(it) if c.get("address") is not None else -1
        for k, c in enumerate(changes):
            r[k]["source"] = next(it) if c.get("source") is not None else -1
            r[k]["incarnation"] = _inc(c.get("incarnationNumber"))
            r[k]["source_incarnation"] = _inc(c.get("sourceIncarnationNumber"))
            r[k]["status"] = STATUS_CODE[c["status"]]
            r[k]["piggyback"] = -1
        return r

    def change(self, row, with_count=False):
        c = {}
        if row["source"] >= 0:
            c["source"] = self.names[row["source"]]
        if row["source_incarnation"] >= 0:
            c["sourceIncarnationNumber"] = int(row["source_incarnation"])
        c["address"] = self.names[row["address"]]
        c["status"] = STATUS_NAME[int(row["status"])]
        c["incarnationNumber"] = int(row["incarnation"])
        if with_count and row["piggyback"] >= 0:
            c["piggybackCount"] = int(row["piggyback"])
        return c


class Membership:
    """lib/membership.js:31-354 on the device.  `ready` stands for
    ringpop.isReady (update() stashes until then, :218-224); `on_updated` /
    `on_set` receive the applied / set updates, as the 'updated' and 'set'
    listeners do (lib/membership-update-listener.js,
    lib/membership-set-listener.js)."""

    def __init__(self, node, ready=False, now=None, on_updated=None, on_set=None):
        self.node = node
        self.isReady = ready
        self.checksum = None
        self.stashedUpdates = []
        self.localMember = None
        self._now = now or (lambda: 0)
        self.on_updated, self.on_set = on_updated, on_set

    def whoami(self):
        return self.node.names[0]

    # :208-313
    def update(self, changes, is_local=False):
        changes = changes if isinstance(changes, list) else [changes]
        if not changes:
            return []
        if not is_local and not self.isReady:
            if isinstance(self.stashedUpdates, list):
                self.stashedUpdates.append(changes)
            return []
        rows = self.node.rows(changes)
        applied = np.zeros(len(changes), dtype=np.uint8)
        na, cs = ctypes.c_uint32(0), ctypes.c_uint32(0)
        check(lib().rp_membership_update(self.node._h, ptr(rows), len(changes), ctypes.c_uint64(self._now()),
                                         ptr(applied), ctypes.byref(na), ctypes.byref(cs)))
        updates = []
        for k, c in enumerate(changes):
            if not applied[k]:
                continue
            if (rows[k]["incarnation"] != _inc(c.get("incarnationNumber"))
                    or int(rows[k]["status"]) != STATUS_CODE[c["status"]]):  # _.extend(change, assertion), :246-251
                c["status"] = STATUS_NAME[int(rows[k]["status"])]
                c["incarnationNumber"] = int(rows[k]["incarnation"])
            if c.get("address") == self.whoami() and self.localMember is None:
                self.localMember = c["address"]
            updates.append(c)
        if updates:
            self.checksum = cs.value
            if self.on_updated:
                self.on_updated(updates)
        return updates

    # :162-206
    def set(self):
        if self.isReady or self.stashedUpdates is None:
            return
        if not isinstance(self.stashedUpdates, list) or not self.stashedUpdates:
            return
        flat = [c for cs in self.stashedUpdates for c in cs]
        rows = self.node.rows(flat)
        win = np.zeros(max(len(flat), 1), dtype=np.uint32)
        nw, cs = ctypes.c_uint32(0), ctypes.c_uint32(0)
        check(lib().rp_membership_set(self.node._h, ptr(rows), len(flat), ptr(win), ctypes.byref(nw),
                                      ctypes.byref(cs)))
        updates = [flat[i] for i in win[: nw.value].tolist()]
        self.stashedUpdates = None
        self.checksum = cs.value
        if self.on_set:
            self.on_set(updates)

    def _make(self, address, incarnation, status, is_local=None):
        # makeUpdate (:324-352)
        lm = self.findMemberByAddress(self.localMember) if self.localMember else None
        if lm is None:
            lm = {"address": address, "incarnationNumber": incarnation}
        return self.update({"source": lm["address"], "sourceIncarnationNumber": lm["incarnationNumber"],
                            "address": address, "status": status, "incarnationNumber": incarnation,
                            "timestamp": self._now()}, is_local)

    def makeAlive(self, address, incarnation):
        return self._make(address, incarnation, "alive", address == self.whoami())

    def makeSuspect(self, address, incarnation):
        return self._make(address, incarnation, "suspect")

    def makeFaulty(self, address, incarnation):
        return self._make(address, incarnation, "faulty")

    def makeLeave(self, address, incarnation):
        return self._make(address, incarnation, "leave")

    @property
    def members(self):
        cnt = ctypes.c_uint32(0)
        check(lib().rp_membership_members(self.node._h, None, None, None, 0, ctypes.byref(cnt)))
        n = cnt.value
        ids = np.zeros(max(n, 1), dtype=np.uint32)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        inc = np.zeros(max(n, 1), dtype=np.uint64)
        check(lib().rp_membership_members(self.node._h, ptr(ids), ptr(st), ptr(inc), max(n, 1), ctypes.byref(cnt)))
        return [{"address": self.node.names[i], "status": STATUS_NAME[int(s)], "incarnationNumber": int(x)}
                for i, s, x in zip(ids[:n].tolist(), st[:n].tolist(), inc[:n].tolist())]

    def findMemberByAddress(self, address):
        for m in self.members:
            if m["address"] == address:
                return m
        return None

    def getMemberCount(self):
        cnt = ctypes.c_uint32(0)
        check(lib().rp_membership_members(self.node._h, None, None, None, 0, ctypes.byref(cnt)))
        return cnt.value

    def getIncarnationNumber(self):
        m = self.findMemberByAddress(self.localMember) if self.localMember else None
        return m and m["incarnationNumber"]

    def isPingable(self, member):
        return member["address"] != self.whoami() and member["status"] in ("alive", "suspect")

    def getRandomPingableMembers(self, n, excluding):
        """:111-120 with underscore 1.13 sample(list, n) on the instance's Math.random."""
        f = [m for m in self.members if m["address"] not in excluding and self.isPingable(m)]
        k = min(n, len(f))
        draws = self.random(k)
        for i in range(k):
            r = i + int(np.floor(draws[i] * (len(f) - i)))
            f[i], f[r] = f[r], f[i]
        return f[:k]

    def random(self, k):
        out = np.zeros(max(k, 1), dtype=np.float64)
        if k:
            check(lib().rp_membership_random(self.node._h, k, ptr(out)))
        return out[:k]

    def computeChecksum(self):
        cs = ctypes.c_uint32(0)
        check(lib().rp_membership_checksum(self.node._h, ctypes.byref(cs)))
        self.checksum = cs.value
        return self.checksum

    def generateChecksumString(self):
        n = ctypes.c_size_t(0)
        check(lib().rp_membership_checksum_string(self.node._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        check(lib().rp_membership_checksum_string(self.node._h, buf, n.value + 1, ctypes.byref(n)))
        return buf.raw[: n.value].decode()

    def shuffle(self):
        check(lib().rp_membership_shuffle(self.node._h))

    def force(self, address, status, incarnation):
        """Set a member's fields directly (what the reference's tests do to Member objects)."""
        check(lib().rp_membership_force(self.node._h, self.node.ids[address], STATUS_CODE[status],
                                        ctypes.c_uint64(incarnation)))


class Dissemination:
    """lib/dissemination.js:27-184 on the device (the instance's change table)."""
    Defaults = {"maxPiggybackCount": 1, "piggybackFactor": 15}

    def __init__(self, node, membership=None):
        self.node = node
        self.membership = membership
        self.maxPiggybackCount = self.Defaults["maxPiggybackCount"]
        self.piggybackFactor = self.Defaults["piggybackFactor"]

    def adjustMaxPiggybackCount(self, server_count):
        """:38-55: piggybackFactor * ceil(log10(serverCount + 1)) (exact integer rule)."""
        x, digits, p = server_count + 1, len(str(server_count + 1)), 10 ** (len(str(server_count + 1)) - 1)
        self.maxPiggybackCount = self.piggybackFactor * (digits - 1 if x == p else digits)

    def resetMaxPiggybackCount(self):
        self.maxPiggybackCount = self.Defaults["maxPiggybackCount"]

    def recordChange(self, change):
        self.recordChanges([change])

    def recordChanges(self, changes):
        if changes:
            rows = self.node.rows(changes)
            check(lib().rp_dissemination_record(self.node._h, ptr(rows), len(changes)))

    def _cap(self):
        cnt = ctypes.c_uint32(0)
        check(lib().rp_dissemination_changes(self.node._h, None, 0, ctypes.byref(cnt)))
        return max(cnt.value, self.membership.getMemberCount() if self.membership else 0, 1)

    def issueAsSender(self):
        out = np.zeros(self._cap(), dtype=ROW)
        cnt = ctypes.c_uint32(0)
        check(lib().rp_dissemination_issue(self.node._h, self.maxPiggybackCount, ptr(out), len(out),
                                           ctypes.byref(cnt)))
        return [self.node.change(r) for r in out[: cnt.value]]

    def issueAsReceiver(self, sender_addr, sender_inc, sender_checksum):
        out = np.zeros(self._cap(), dtype=ROW)
        cnt, fs = ctypes.c_uint32(0), ctypes.c_int(0)
        src = self.node.intern([sender_addr])[0] if sender_addr else -1
        inc = -1 if not sender_inc else _inc(sender_inc)
        check(lib().rp_dissemination_issue_as_receiver(
            self.node._h, src, inc, ctypes.c_uint32((sender_checksum or 0) & 0xFFFFFFFF),
            0 if sender_checksum is None else 1, self.maxPiggybackCount, ptr(out), len(out), ctypes.byref(cnt),
            ctypes.byref(fs)))
        self.last_full_sync = bool(fs.value)
        return [self.node.change(r) for r in out[: cnt.value]]

    def fullSync(self):
        n = self._cap()
        out = np.zeros(n, dtype=ROW)
        cnt = ctypes.c_uint32(0)
        check(lib().rp_dissemination_full_sync(self.node._h, ptr(out), n, ctypes.byref(cnt)))
        return [self.node.change(r) for r in out[: cnt.value]]

    def clearChanges(self):
        check(lib().rp_dissemination_clear(self.node._h))

    @property
    def changes(self):
        """{address: change} in key order, with piggybackCount where defined."""
        cnt = ctypes.c_uint32(0)
        check(lib().rp_dissemination_changes(self.node._h, None, 0, ctypes.byref(cnt)))
        out = np.zeros(max(cnt.value, 1), dtype=ROW)
        check(lib().rp_dissemination_changes(self.node._h, ptr(out), len(out), ctypes.byref(cnt)))
        return {self.node.names[r["address"]]: self.node.change(r, True) for r in out[: cnt.value]}
