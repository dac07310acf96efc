#!/bin/bash
# parity + bench + issue section cycles after the prologue / prefix-pack rework
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
for v in f1:1 f2:2; do
  b=${v%%:*}; ph=${v##*:}
  RP_DIAG_FINE=1 RP_DIAG_PHASE=$ph RINGPOP_HIP_LIB=$PWD/ringpop_amd/variants/libringpop_hip_$b.so timeout -k 10 300 python3 -u tools/diag.py 65536 > gpurun_out/diag_$b.json 2>&1 || { echo $b failed; tail -3 gpurun_out/diag_$b.json; exit 1; }
  echo "== $b"; cat gpurun_out/diag_$b.json
done
