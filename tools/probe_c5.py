"""Per-round counter deltas of config 5 (experiments only).

python tools/probe_c5.py [nodes] [shards]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ringpop_amd as rp  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
G = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nf = -(-N // 10)
dead = np.sort(np.random.default_rng(2024).choice(N, size=nf, replace=False))
kw = {"arena_entries": (N // G) * 32768} if G > 1 else {}
S = rp.Sim(N, 2024, churn_k=0, failures={0: dead.tolist()}, storm={"start": 0, "end": 20, "ppm": 1000}, shards=G, **kw)
keys = ("evaluated", "touched", "applied", "checksum_views", "written_send_issue", "written_recv_issue", "emitted_send_issue",
        "emitted_recv_issue", "full_syncs", "messages")
prev = S.counters()
tot = {k: 0 for k in keys}
print("round ms " + " ".join(keys), flush=True)
for r in range(int(sys.argv[3]) if len(sys.argv) > 3 else 60):
    S.sync()
    t0 = time.perf_counter()
    st = S.round(churn=False)
    S.sync()
    ms = (time.perf_counter() - t0) * 1e3
    c = S.counters()
    d = {k: c[k] - prev[k] for k in keys}
    prev = c
    for k in keys:
        tot[k] += d[k]
    print(r, f"{ms:.2f}", " ".join(str(d[k]) for k in keys), int(st["converged"]), flush=True)
print("total", tot)
S.close()
