#!/bin/bash
# config-3 lookup bench for the default build and each variant named as an argument
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for v in default "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload lookup --no-cpu-baseline > gpurun_out/lk_$v.json 2> gpurun_out/lk_$v.err
  rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/lk_$v.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['parity'])" || { echo "$v failed rc=$rc"; tail -3 gpurun_out/lk_$v.err; exit 1; }
done
