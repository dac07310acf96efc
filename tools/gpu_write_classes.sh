#!/bin/bash
# WRITE_SIZE per launch of the merge kernels for library variants that each
# drop one store class of wg_apply (measurement only: the variants diverge
# from the reference after their first round).  Variants are built by
# tools/build_variant.sh; "default" is the in-tree library.
# usage: tools/gpu_write_classes.sh tag variant...
set -u
TAG=$1; shift
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L bash tools/traffic.sh 65536 10 5 ${TAG}_$v > /dev/null || { echo "$v failed"; exit 1; }
  echo "== $v"
  python3 -c "
import json; d = json.load(open('gpurun_out/traffic_${TAG}_$v/traffic_${TAG}_$v.json'))
for k, x in d.items():
    if 'write_kib' in x: print(f\"{k:14s} x{x['launches_per_round']} fetch*2 {2*x['fetch_kib_raw']*1024/1e9:.3f} GB  write {x['write_kib']*1024/1e9:.3f} GB per launch\")
"
done
