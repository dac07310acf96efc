"""Section cycle shares of the RP_DIAG build (build.py --diag): phase-2
issue (flags incl. seen lookups, rank exchange, stores) and phase-2 apply vs
respond, per round at full size.  Run with RINGPOP_HIP_LIB pointing at
libringpop_hip_diag.so."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ringpop_amd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
k = math.ceil(0.01 * n)
S = ringpop_amd.Sim(n, 2024, churn_k=k)
S.run(20)
S.sync()
c0 = S.counters()
S.run(5)
S.sync()
c1 = S.counters()
d = {key: (c1[key] - c0[key]) / 5 for key in c1}
names = {"diag0": "p2 issue: pass 1 (stream, flags)", "diag1": "p2 issue: exchange + pass 2 (gather, stores)",
         "diag2": "p2 issue: prologue (scalars, seen staging, arena reservation)", "diag3": "p2 apply (merge)",
         "diag4": "p2 issue: epilogue (reductions, node scalars)", "diag5": "p2 respond total (issue + record)"}
pings = d["pings"]
if os.environ.get("RP_DIAG_PHASE") == "1":  # (a build with -DRP_DIAG_PHASE=1: issueAsSender sections)
    names = {"diag0": "p1 issue: pass 1 (stream, flags)", "diag1": "p1 issue: exchange + pass 2 (gather, stores)",
             "diag2": "p1 issue: prologue (scalars, seen staging, arena reservation)", "diag3": "(p2 apply)",
             "diag4": "p1 issue: epilogue (reductions, prefix packing, node scalars)", "diag5": "(p2 respond)"}
if os.environ.get("RP_DIAG_FINE") == "1":  # (-DRP_DIAG_FINE=1: the issue's prologue and epilogue split)
    ph = "p" + os.environ.get("RP_DIAG_PHASE", "2")
    names = {"diag0": ph + " issue: prologue to its barrier (thread 0 scalars, same-view check)",
             "diag1": ph + " issue: prologue barrier wait", "diag2": ph + " issue: block reductions",
             "diag3": ph + " issue: node scalars + barrier", "diag4": ph + " issue: prefix packing",
             "diag5": ph + " issue: passes 1 and 2"}
print(json.dumps({names[k] + " per ping": round(d[k] / pings) for k in names}, indent=1))
