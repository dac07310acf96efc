#!/bin/bash
# per-round GPU busy/idle of config 5 at 65,536 nodes on 4 in-process shards
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -s KILL 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/rg64 -o run -- python3 tools/probe_c5.py 65536 4 > gpurun_out/rg64.log 2>&1 || { echo trace failed; tail -3 gpurun_out/rg64.log; exit 1; }
for r in "3 12" "20 29" "30 39" "45 55"; do set -- $r
  python3 tools/round_gaps.py gpurun_out/rg64 k_seen_clear 4 --from $1 --to $2 > gpurun_out/round_gaps64_$1.txt
done
head -16 gpurun_out/round_gaps64_30.txt
find gpurun_out/rg64 -name "*.csv" -size +20M -delete
cat gpurun_out/rg64.log | head -70
