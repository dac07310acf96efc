#!/bin/bash
# exchange-buffer growth events of config 5 at 65,536 nodes on 4 in-process shards
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
RP_DEBUG_GROW=1 timeout -k 10 300 python3 -u tools/probe_c5.py 65536 4 > gpurun_out/grow64.log 2>&1 || { echo probe failed; tail -3 gpurun_out/grow64.log; exit 1; }
grep -c grow gpurun_out/grow64.log; grep grow gpurun_out/grow64.log | awk '{t+=$(NF-1)} END {print "total grow ms", t}'; head -60 gpurun_out/grow64.log
