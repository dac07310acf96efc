"""Per-launch HBM bytes of each kernel over the last K dispatches (the bench's
timed region) from tools/traffic.sh's FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md,
HBM section): FETCH_SIZE reports half the bytes of 16-B-per-lane streaming
reads.  Calibrated for this path's other access kinds too
(tools/micro/fetch_cal.hip, profiles/r04/fetch_cal_r04n.json): a random 16-B or
4-B read reports 60 B (a 128-B line, halved), a 4-B-per-lane stream half its
bytes, and WRITE_SIZE a 32-B sector per partial write -- so hbm = 2 * FETCH +
WRITE holds for every kind the round kernels use."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, last = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20


def per_dispatch(sub, counter):
    vals = defaultdict(dict)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            # "void rp::k_phase2<false>(...)" -> "k_phase2"
            k = r["Kernel_Name"].split("(")[0].replace("rp::", "").replace("void ", "").split("<")[0]
            did = int(r["Dispatch_Id"])
            vals[k][did] = vals[k].get(did, 0.0) + float(r["Counter_Value"])
    # launches per round: relative to k_phase1 (one launch per round)
    per_round = {k: max(1, round(len(v) / max(len(vals.get("k_phase1", v)), 1))) for k, v in vals.items()}
    return {k: [v[i] for i in sorted(v)][-last * per_round[k]:] for k, v in vals.items()}, per_round


(fetch, per_round), (write, _) = per_dispatch("fetch", "FETCH_SIZE"), per_dispatch("write", "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, []), write.get(k, [])
    fk = sum(f) / max(len(f), 1)
    wk = sum(w) / max(len(w), 1)
    out[k] = {"dispatches": len(f), "launches_per_round": per_round.get(k, 1), "fetch_kib_raw": round(fk, 1),
              "write_kib": round(wk, 1), "hbm_bytes_per_launch": int((2 * fk + wk) * 1024),
              "note": "2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes"}
# the ping-merge stage (bench.py's roofline kernel): its launches of one round
stage = [k for k in ("k_p2_apply", "k_p2_respond", "k_phase2") if k in out]
if "k_p2_apply" in out:
    out["k_phase2 stage"] = {"kernels": stage, "hbm_bytes_per_round": int(sum(
        out[k]["hbm_bytes_per_launch"] * out[k]["launches_per_round"] for k in stage))}
print(json.dumps(out, indent=1))
