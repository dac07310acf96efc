#!/bin/bash
# config 5 (single shard): bench line, then a rocprofv3 kernel-trace + stats of the same run
set -u
TAG=${1:-c5}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --workload failure > gpurun_out/failure_$TAG.json 2> gpurun_out/failure_$TAG.err
rc=$?; echo "failure exit $rc"; cat gpurun_out/failure_$TAG.json; tail -2 gpurun_out/failure_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- python3 bench.py --workload failure > gpurun_out/prof_$TAG/trace.log 2>&1
rc=$?; echo "trace exit $rc"; head -16 gpurun_out/prof_$TAG/trace/run_kernel_stats.csv | cut -d, -f1-4; exit $rc
