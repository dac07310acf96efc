"""The two checksum paths on config 4's views (65,536 nodes, 656 re-assertions
per round): after a pre-roll, each measured round is followed by a read of
every node's checksum (tick-cluster's check, scripts/tick-cluster.js:88-115);
ms of that read, the distinct views hashed, per path.
usage: python tools/ck_paths.py [nodes] [preroll] [reads]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import ringpop_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
pre = int(sys.argv[2]) if len(sys.argv) > 2 else 30
reads = int(sys.argv[3]) if len(sys.argv) > 3 else 3
out = {}
ref = None
modes = [("lanes", 1), ("waves", 0xFFFFFFFF), ("auto", 0)]
want = os.environ.get("CK_MODES")
if want:
    modes = [m for m in modes if m[0] in want.split(",")]
for mode, lane_min in modes:
    S = ringpop_amd.Sim(n, 2024, churn_k=-(-n // 100), ck_lane_min=lane_min)
    S.run(pre)
    S.sync()
    rows = []
    for _ in range(reads):
        S.round(churn=True)
        S.sync()
        c0 = S.counters()["checksum_views"]
        t0 = time.perf_counter()
        cs = S.checksums()
        ms = (time.perf_counter() - t0) * 1e3
        rows.append({"ms": round(ms, 2), "views_hashed": S.counters()["checksum_views"] - c0,
                     "distinct": int(len(np.unique(cs)))})
    if ref is None:
        ref = cs
    assert np.array_equal(cs, ref), mode
    out[mode] = rows
    S.close()
    print(mode, rows, file=sys.stderr, flush=True)
print(json.dumps(out))
