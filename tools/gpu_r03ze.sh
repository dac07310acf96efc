#!/bin/bash
# parity + two bench runs of the current tree
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py > gpurun_out/bench$i.json 2> gpurun_out/bench$i.err || { echo bench failed; tail -5 gpurun_out/bench$i.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench$i.json'))
print(d['ms_per_step'],d['kernel_ms'],{k:v['avg_launch_ms'] for k,v in d['stages'].items()}, d['config5']['ms_per_step'])"
done
