"""Per-round load of config 4 from a fresh start: evaluated / touched /
applied changes and device ms per round, to place bench.py's pre-roll at the
steady state.  usage: python tools/steady_probe.py [rounds] [nodes]"""
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ringpop_amd  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 120
N = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
S = ringpop_amd.Sim(N, 2024, churn_k=math.ceil(0.01 * N))
rows, prev = [], S.counters()
for r in range(R):
    t = time.perf_counter()
    S.run(1)
    S.sync()
    dt = time.perf_counter() - t
    c = S.counters()
    rows.append({"round": r, "ms": round(dt * 1e3, 3), **{k: c[k] - prev[k] for k in
                 ("evaluated", "touched", "applied", "scanned_recv_issue", "written_recv_issue", "full_syncs")}})
    prev = c
    print(json.dumps(rows[-1]), flush=True)
S.close()
