#!/bin/bash
# Round evidence: GPU tests, the default bench line (with CPU baseline),
# rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes.
# usage: tools/gpu_round_evidence.sh <tag>
set -u
TAG=${1:-r01}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
PROFILE_PMC=0 bash tools/profile.sh 65536 20 20 $TAG || exit $?
bash tools/traffic.sh 65536 20 20 $TAG || exit $?
python3 tools/trace_summary.py gpurun_out/prof_$TAG/trace/run_kernel_trace.csv 20 > gpurun_out/prof_$TAG/steady.txt
cat gpurun_out/traffic_$TAG/traffic_$TAG.json
head -8 gpurun_out/prof_$TAG/steady.txt
