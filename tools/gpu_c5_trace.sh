#!/bin/bash
# Config 5 (mass failure + storm) under a rocprofv3 kernel trace: per-kernel
# totals over the run, split by the stream (queue) they ran on, so that the
# checksum work on the side stream and what stays on the round's stream show
# separately.  (No --pmc in this run.)
# usage: tools/gpu_c5_trace.sh tag [bench.py args...]
set -u
TAG=$1; shift
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
PY=$(command -v python3)  # (an absolute path after rocprofv3's --)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5tr_$TAG -o run --output-format csv -- "$PY" bench.py \
    --workload failure --no-cpu-baseline "$@" > gpurun_out/c5tr_$TAG.log 2>&1
rc=$?; echo "rocprofv3 exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/c5tr_$TAG.log; exit $rc; }
python3 - "$TAG" > gpurun_out/c5tr_$TAG.txt <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(f"gpurun_out/c5tr_{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
qkey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
agg = defaultdict(lambda: [0, 0])
perq = defaultdict(int)
for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    k = r["Kernel_Name"].split("(")[0].replace("rp::", "").replace("void ", "")
    agg[(r[qkey], k)][0] += d
    agg[(r[qkey], k)][1] += 1
    perq[r[qkey]] += d
print(f"{qkey}: total kernel ms", {q: round(t / 1e6, 2) for q, t in perq.items()})
for (q, k), (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:45]:
    print(f"{q:>4s} {k[:56]:56s} {c:6d} {t / 1e6:9.2f} ms {t / c / 1e3:9.1f} us")
PY
cat gpurun_out/c5tr_$TAG.txt | head -30
