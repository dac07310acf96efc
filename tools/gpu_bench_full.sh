#!/bin/bash
# headline bench (config 4, 65,536 nodes) then rocprofv3 kernel trace; stop at first failure
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_full.json; tail -5 gpurun_out/bench_full.err
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh 65536 5 20 r01_trace_only 2>&1 | head -1
