#!/bin/bash
# Consecutive bench processes on one box (the k_phase3 / k_p2_apply "slow
# mode" alternates between processes): per run, whether rp_calibrate ran
# first (cal / nocal), the merge kernels' mean times and ms/round.
# usage: tools/gpu_mode_probe.sh cal|nocal ...
set -u
PY=$(command -v python3)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for m in "$@"; do
  i=$((i + 1))
  if [ "$m" = nocal ]; then export RP_BENCH_NO_CAL=1; else unset RP_BENCH_NO_CAL; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mp_$i -o run --output-format csv -- "$PY" bench.py \
      --steps 10 --no-cpu-baseline --no-extras --no-traffic > gpurun_out/mp_$i.log 2>&1 || { echo "run $i failed"; tail -5 gpurun_out/mp_$i.log; exit 1; }
  python3 - "$i" "$m" <<'PY'
import csv, glob, re, sys
i, m = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/mp_{i}/**/run_kernel_stats.csv", recursive=True)[0]
t = {r["Name"].split("(")[0].replace("void ", "").replace("rp::", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
ms = re.findall(r'"ms_per_step": ([0-9.]+)', open(f"gpurun_out/mp_{i}.log").read())
print(i, m, {k: round(v, 1) for k, v in t.items() if k.startswith(("k_phase3<", "k_p2_apply", "k_phase1<"))}, ms[:1])
PY
done
