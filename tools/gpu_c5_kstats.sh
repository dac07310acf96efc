#!/bin/bash
# Per-kernel rocprof means of config 5 (bench.py --workload failure) for each
# library variant given (tools/build_variant.sh; "default" = the in-tree build).
# usage: tools/gpu_c5_kstats.sh variant...
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
PY=$(command -v python3)
lib_of() { if [ "$1" = default ]; then echo "$PWD/ringpop_amd/libringpop_hip.so"; else echo "$PWD/ringpop_amd/variants/libringpop_hip_$1.so"; fi; }
i=0
for v in "$@"; do
  i=$((i+1))
  RINGPOP_HIP_LIB=$(lib_of $v) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5k_${i}_$v -o run --output-format csv -- "$PY" bench.py --workload failure --no-cpu-baseline --no-extras --no-traffic ${C5_ARGS:-} > gpurun_out/c5k_${i}_$v.json 2> gpurun_out/c5k_${i}_$v.err || { echo "$v failed"; tail -3 gpurun_out/c5k_${i}_$v.err; exit 1; }
  echo "== $v $(python3 -c "import json; d = json.load(open('gpurun_out/c5k_${i}_$v.json')); print(d['value'], d['ms_per_step'])")"
  python3 - gpurun_out/c5k_${i}_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if not r["Name"].startswith(("rp::k_shuffle", "rp::k_init", "rp::k_view_counts"))]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f"  {r['Name'][:52]:52s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
