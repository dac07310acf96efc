#!/bin/bash
# Round 6: where the sharded rounds' extra device time goes, and the single
# shard's launch list.  (1) 8 loopback ranks of config 4 (tools/gpu_gaps.sh:
# busy/idle per round, per-kernel time); (2) rocprofv3 --kernel-trace --stats
# of the one-shard headline bench (launches per round); (3) config 4 on 4
# in-process shards.
# usage: tools/gpu_r06_shard.sh TAG
set -u
TAG=$1
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
PY=$(command -v python3)
bash tools/gpu_gaps.sh loop8_$TAG 8 65536 10 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- "$PY" bench.py \
    --steps 20 --no-cpu-baseline --no-extras --no-traffic > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$TAG.log; exit $rc; }
python3 tools/trace_summary.py $(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1) 20 > gpurun_out/prof_$TAG.txt 2>&1 || true
timeout -k 10 300 python -u bench.py --shards 4 --no-extras --no-cpu-baseline --no-traffic > gpurun_out/bench_sh4_$TAG.json 2> gpurun_out/bench_sh4_$TAG.err
rc=$?; echo "shards4 exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_sh4_$TAG.err; exit $rc; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_sh4_$TAG.json | head -1
