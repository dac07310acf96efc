"""Summarise tools/pmc.sh output: per kernel, the counters of the last K
dispatches (steady-state rounds), averaged per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch]
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    per = defaultdict(lambda: defaultdict(float))
    times = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        per[(k, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
        times[(k, int(r["Dispatch_Id"]))] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    byk = defaultdict(list)
    for (k, did) in per:
        byk[k].append(did)
    for k, ids in byk.items():
        for did in sorted(ids)[-last:]:
            for c, v in per[(k, did)].items():
                vals[k][c].append(v)
            dur[k].append(times[(k, did)])
for k in sorted(vals):
    print(k, f"(mean dispatch under counters {sum(dur[k]) / len(dur[k]) / 1e6:.2f} ms)")
    for c in sorted(vals[k]):
        v = vals[k][c]
        print(f"   {c:24s} {sum(v) / len(v):16.4e}")
