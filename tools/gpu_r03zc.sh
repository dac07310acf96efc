#!/bin/bash
# wg_issue section cycles at 65,536 nodes (RP_DIAG builds, finer split)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for v in f1:1 f2:2 f1n:1; do
  b=${v%%:*}; ph=${v##*:}
  RP_DIAG_FINE=1 RP_DIAG_PHASE=$ph RINGPOP_HIP_LIB=$PWD/ringpop_amd/variants/libringpop_hip_$b.so timeout -k 10 300 python3 -u tools/diag.py 65536 > gpurun_out/diag_$b.json 2>&1 || { echo $b failed; tail -3 gpurun_out/diag_$b.json; exit 1; }
  echo "== $b"; cat gpurun_out/diag_$b.json
done
