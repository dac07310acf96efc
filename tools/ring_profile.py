"""Where a single addServer / removeServer goes: the
benchmark's pattern (benchmarks/add-remove-hashring.js:35-52: 1,000 servers of
large-membership.json added one at a time, then removed one at a time), each
call followed by the ring checksum as HashRing.addServer does
(lib/ring.js:39-58,96-105), through the C ABI.  Per call: the host phases of
rp_ring_add_remove and rp_ring_checksum (rp_ring_profile), the device time of
the update (rp_ring_build_ms: HIP events around its device work) and the host
wall clock of the pair.

usage: python tools/ring_profile.py [reps]   (GPU box)"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import ringpop_amd  # noqa: E402
from ringpop_amd._lib import check, lib  # noqa: E402

PHASES = ["select", "hash", "merge", "index", "total", "ck_build", "ck_hash"]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    recs = json.load(open(os.path.join(ROOT, "tests", "golden", "large_membership_input.json")))[:1000]
    servers = [r["address"] for r in recs]
    L = lib()
    ring = ringpop_amd.HashRing()
    prof = (ctypes.c_double * len(PHASES))()
    dev = ctypes.c_double(0)
    acc = {k: [] for k in PHASES + ["device_update", "wall_pair", "wall_add_remove", "wall_checksum"]}

    enc = {s: (np.frombuffer(s.encode() + b"\0", dtype=np.uint8), np.array([0, len(s)], dtype=np.uint64))
           for s in servers}
    changed, cs = ctypes.c_int(0), ctypes.c_uint32(0)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731

    def one(add, name):
        b, o = enc[name]
        t0 = time.perf_counter()
        if add:
            check(L.rp_ring_add_remove(ring._h, P(b), P(o), 1, None, None, None, 0, None, ctypes.byref(changed)))
        else:
            check(L.rp_ring_add_remove(ring._h, None, None, 0, None, P(b), P(o), 1, None, ctypes.byref(changed)))
        t1 = time.perf_counter()
        check(L.rp_ring_checksum(ring._h, ctypes.byref(cs)))
        t2 = time.perf_counter()
        check(L.rp_ring_profile(ring._h, prof, len(PHASES)))
        check(L.rp_ring_build_ms(ring._h, ctypes.byref(dev)))
        return t1 - t0, t2 - t1

    for r in range(reps + 1):
        for add in (True, False):
            for s in servers:
                a, c = one(add, s)
                if r == 0:
                    continue  # (warm-up pass)
                for i, k in enumerate(PHASES):
                    acc[k].append(prof[i])
                acc["device_update"].append(dev.value * 1e3)
                acc["wall_add_remove"].append(a * 1e6)
                acc["wall_checksum"].append(c * 1e6)
                acc["wall_pair"].append((a + c) * 1e6)
    out = {"servers": len(servers), "reps": reps, "calls": len(acc["total"]), "unit": "us per call (median, mean)",
           "phases": {k: [round(float(np.median(v)), 2), round(float(np.mean(v)), 2)] for k, v in acc.items()},
           "note": "select/hash/merge/index/total: host phases of rp_ring_add_remove (incremental path); "
                   "ck_build/ck_hash: rp_ring_checksum's host string and its device hash incl. sync; "
                   "device_update: HIP events around the update's device work; wall_*: Python wall clock "
                   "(ctypes marshalling included)"}
    ring.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
