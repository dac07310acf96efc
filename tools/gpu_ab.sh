#!/bin/bash
# A/B of library variants (tools/build_variant.sh; "default" = the in-tree
# build): per variant the headline bench's per-kernel rocprof means
# (tools/gpu_kstats.sh) and, with AB_PMC=1, the round kernels' FETCH/WRITE
# bytes per round (tools/traffic.sh; separate --pmc passes).
# usage: tools/gpu_ab.sh name ...
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
bash tools/gpu_kstats.sh "$@" || exit $?
[ "${AB_PMC:-0}" = 1 ] || exit 0
for v in "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L bash tools/traffic.sh 65536 10 5 ab_$v > /dev/null || { echo "$v pmc failed"; exit 1; }
  echo "== $v traffic"
  python3 -c "
import json; d = json.load(open('gpurun_out/traffic_ab_$v/traffic_ab_$v.json'))
for k, x in d.items():
    if 'fetch_kib_raw' in x: print(f\"{k:14s} x{x['launches_per_round']} fetch*2 {2*x['fetch_kib_raw']*1024/1e9:.3f} GB  write {x['write_kib']*1024/1e9:.3f} GB per launch\")
"
done
