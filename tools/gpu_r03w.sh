#!/bin/bash
# per-round counters of config 5 at 65,536 nodes on 1 and 4 shards (current tree)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/probe_c5.py 65536 1 > gpurun_out/probe64_sh1.log 2>&1 || { echo probe1 failed; tail -3 gpurun_out/probe64_sh1.log; exit 1; }
timeout -k 10 300 python3 -u tools/probe_c5.py 65536 4 > gpurun_out/probe64_sh4.log 2>&1 || { echo probe4 failed; tail -3 gpurun_out/probe64_sh4.log; exit 1; }
paste -d' ' <(awk '{print $1, $2, $4, $5}' gpurun_out/probe64_sh1.log) <(awk '{print $2, $4, $5}' gpurun_out/probe64_sh4.log) | head -62
