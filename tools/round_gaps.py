"""Per-round split of wall time into GPU-busy and idle, with the host API
calls that fill the idle time, from rocprofv3 CSVs (experiments only).

usage: round_gaps.py <dir with run_kernel_trace.csv [run_hip_api_trace.csv]
                      [run_memory_copy_trace.csv]> <boundary kernel> <launches per round>
                      [--from ROUND] [--to ROUND]
Rounds are delimited by every <launches per round>-th launch of the boundary
kernel (e.g. k_round_start, one per shard per round).
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d, name):
    f = glob.glob(f"{d}/**/*{name}.csv", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


d, bk, per = sys.argv[1], sys.argv[2], int(sys.argv[3])
r_from = int(sys.argv[sys.argv.index("--from") + 1]) if "--from" in sys.argv else 0
r_to = int(sys.argv[sys.argv.index("--to") + 1]) if "--to" in sys.argv else 10 ** 9
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("rp::", ""))
      for r in load(d, "kernel_trace")]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?"))
       for r in load(d, "memory_copy_trace")]
ev.sort()
api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in load(d, "hip_api_trace")]
api.sort()
starts = [s for s, _, k in ev if k.startswith(bk)][::per]
starts.append(ev[-1][1])
print(f"{len(starts) - 1} rounds delimited by {bk}")
agg_k = defaultdict(lambda: [0, 0])
agg_api = defaultdict(lambda: [0, 0])
tot_wall = tot_busy = 0
nr = 0
print(f"{'round':>5s} {'wall_ms':>8s} {'busy_ms':>8s} {'idle_ms':>8s} {'ops':>6s} {'gaps>20us':>9s}")
for r in range(len(starts) - 1):
    lo, hi = starts[r], starts[r + 1]
    if r < r_from or r > r_to:
        continue
    sel = [e for e in ev if lo <= e[0] < hi]
    busy, cs, ce, ng = 0, None, None, 0
    for s, e, k in sel:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
                ng += (s - ce) > 20000
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
    wall = hi - lo
    print(f"{r:5d} {wall / 1e6:8.2f} {busy / 1e6:8.2f} {(wall - busy) / 1e6:8.2f} {len(sel):6d} {ng:9d}")
    tot_wall += wall
    tot_busy += busy
    nr += 1
    for s, e, k in sel:
        agg_k[k][0] += e - s
        agg_k[k][1] += 1
    for s, e, f in api:
        if lo <= s < hi:
            agg_api[f][0] += e - s
            agg_api[f][1] += 1
if nr:
    print(f"mean over {nr} rounds: wall {tot_wall / nr / 1e6:.3f} ms, busy {tot_busy / nr / 1e6:.3f} ms")
    print(f"\n{'kernel/copy':44s} {'per_round':>9s} {'us/round':>9s}")
    for k, (t, c) in sorted(agg_k.items(), key=lambda x: -x[1][0])[:40]:
        print(f"{k[:44]:44s} {c / nr:9.1f} {t / nr / 1e3:9.1f}")
    if agg_api:
        print(f"\n{'host API':44s} {'per_round':>9s} {'us/round':>9s}")
        for k, (t, c) in sorted(agg_api.items(), key=lambda x: -x[1][0])[:25]:
            print(f"{k[:44]:44s} {c / nr:9.1f} {t / nr / 1e3:9.1f}")
