"""FETCH_SIZE / WRITE_SIZE per access of tools/micro/fetch_cal's kernels:
python tools/fetch_cal.py <fetch_counter_collection.csv> <write_counter_collection.csv> <fetch_cal stdout>
(counters in KiB per dispatch; each kernel dispatched twice)."""
import collections
import csv
import json
import sys


def per_kernel(path, name):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
out = {}
for line in open(sys.argv[3]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    k = d["kernel"]
    f = next((v for kk, v in fetch.items() if kk.endswith(k)), None)
    w = next((v for kk, v in write.items() if kk.endswith(k)), None)
    n = d["accesses_per_launch"]
    out[k] = {"G_accesses_per_s": d["G_accesses_per_s"], "requested_B": d["requested_bytes_per_access"],
              "fetch_raw_B_per_access": round(f * 1024 / n, 2) if f is not None else None,
              "write_raw_B_per_access": round(w * 1024 / n, 2) if w is not None else None}
print(json.dumps(out, indent=1))
