#!/bin/bash
# PMC passes over config 5's checksum kernels in its first rounds (the mass
# failure's thousands of distinct views; tools/probe_c5.py), one counter
# group per rocprofv3 run (kernel trace only), then per dispatch longer than
# 2 ms: duration and counters.
# usage: tools/pmc_c5ck.sh <tag> [kernel-regex] [rounds]
set -u
PY=$(command -v python3)  # (an absolute path after rocprofv3's --)
TAG=${1:-c5ck}; RE=${2:-'k_checksums'}; R=${3:-4}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/pmc_c5ck_$TAG
export TMPDIR=/tmp
PASSES=${PMC_PASSES:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM"}
i=0
IFS='|' read -r -a GROUPS_ <<< "$PASSES"
for P in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex "$RE" --pmc $P -d gpurun_out/pmc_c5ck_$TAG/p$i -o run --output-format csv -- "$PY" tools/probe_c5.py 65536 1 $R > gpurun_out/pmc_c5ck_$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i ($P) exit $rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - gpurun_out/pmc_c5ck_$TAG > gpurun_out/pmc_c5ck_$TAG.txt <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
rows = defaultdict(dict)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    p = os.path.basename(os.path.dirname(f))
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0], int(r["Dispatch_Id"]))
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        per[k]["_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    # dispatches in order, per kernel
    byk = defaultdict(list)
    for (k, did), c in sorted(per.items(), key=lambda x: x[0][1]):
        byk[k].append(c)
    for k, lst in byk.items():
        for j, c in enumerate(lst):
            rows[(k, j)].update({(p, n): v for n, v in c.items()})
for (k, j), c in sorted(rows.items()):
    ms = max(v for (p, n), v in c.items() if n == "_ms")
    if ms < 2:
        continue
    print(f"{k} #{j} {ms:.2f} ms", " ".join(f"{n}={v:.4g}" for (p, n), v in sorted(c.items(), key=lambda x: x[0][1]) if n != "_ms"))
PY
cat gpurun_out/pmc_c5ck_$TAG.txt
