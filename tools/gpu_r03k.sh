#!/bin/bash
# headline bench of the current tree, then per-round host/GPU traces of config 5
# at 32,768 nodes on 1 and 4 in-process shards (tools/round_gaps.py)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r03k.json 2> gpurun_out/bench_r03k.err || { echo bench failed; tail -5 gpurun_out/bench_r03k.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r03k.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline'])"
for s in 1 4; do
  timeout -s KILL 400 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/rg_sh$s -o run -- python3 tools/probe_c5.py 32768 $s > gpurun_out/rg_sh$s.log 2>&1 || { echo trace $s failed; tail -3 gpurun_out/rg_sh$s.log; exit 1; }
  python3 tools/round_gaps.py gpurun_out/rg_sh$s k_seen_clear $s --from 46 --to 58 > gpurun_out/round_gaps_sh$s.txt
  python3 tools/round_gaps.py gpurun_out/rg_sh$s k_seen_clear $s --from 30 --to 40 > gpurun_out/round_gaps_mid_sh$s.txt
  head -20 gpurun_out/round_gaps_sh$s.txt
  rm -rf gpurun_out/rg_sh$s/*/*/*.csv.gz 2>/dev/null
done
