"""Steady-state kernel times from a rocprofv3 --kernel-trace CSV: per kernel,
the mean / min / max duration of its last K dispatches (the bench's timed
rounds), in ms.  usage: trace_summary.py <kernel_trace.csv> [K]"""
import csv
import sys
from collections import defaultdict

path, K = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"].split("(")[0].replace("rp::", "")
    d[k].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
# launches per round relative to k_phase1 (one per round); a kernel's last
# K x that many dispatches are the timed rounds
rounds = len(next((v for k, v in d.items() if "k_phase1" in k), [None])) or 1
rows, stage = [], 0.0
for k, v in d.items():
    v.sort()
    per = max(1, round(len(v) / rounds))
    t = [x for _, x in v[-K * per:]]
    rows.append((sum(t) / len(t), k, len(v), min(t), max(t)))
    if any(s in k for s in ("k_p2_lists", "k_p2_apply", "k_p2_respond", "k_phase2")):
        stage += sum(t) / K
print(f"{'kernel':34s} {'calls':>6s} {'mean_ms':>9s} {'min_ms':>9s} {'max_ms':>9s}")
for m, k, c, lo, hi in sorted(rows, reverse=True):
    print(f"{k:34s} {c:6d} {m:9.4f} {lo:9.4f} {hi:9.4f}")
if stage:
    print(f"ping-merge stage per round (k_p2_lists + k_p2_apply + k_p2_respond + k_phase2): {stage:.4f} ms")
