#!/bin/bash
# Per-kernel rocprofv3 stats of the headline bench for each variant library
# (tools/build_variant.sh; "default" = the in-tree build).
# usage: tools/gpu_kstats.sh name ...
set -u
PY=$(command -v python3)  # (an absolute path after rocprofv3's --: no PATH lookup in the profiled exec)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  export RINGPOP_HIP_LIB=$L
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_$v -o run --output-format csv -- "$PY" bench.py --steps 10 --no-cpu-baseline --no-extras --no-traffic > gpurun_out/ks_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ks_$v.log; exit 1; }
  echo "== $v"
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/ks_{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows:
    if not any(k in r["Name"] for k in ("k_phase", "k_p2_", "k_checksums", "k_pending", "k_iterate", "k_need", "k_churn", "k_shuffle")):
        continue
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:10.1f} us')
PY
  grep -o "\"ms_per_step\": [0-9.]*" gpurun_out/ks_$v.log || true
done
