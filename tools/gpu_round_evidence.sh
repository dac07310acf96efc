#!/bin/bash
# Round evidence in one GPU call: the GPU tests, the default bench line (with
# configs 3 and 5 and the CPU baselines), a rocprofv3 kernel trace + stats of
# the headline, and FETCH_SIZE / WRITE_SIZE passes (separate --pmc runs).
# Every GPU step has its own time limit; a timeout, abort or fault ends the
# script (test assertion failures do not stop the bench).
# usage: tools/gpu_round_evidence.sh <tag> [pytest-args...]
set -u
TAG=${1:-r02}; shift || true
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log; fatal $rc && exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
[ "${NO_PROFILE:-0}" = 1 ] && exit 0
PROFILE_PMC=0 bash tools/profile.sh 65536 20 5 $TAG || exit $?
bash tools/traffic.sh 65536 20 5 $TAG || exit $?
python3 tools/trace_summary.py gpurun_out/prof_$TAG/trace/run_kernel_trace.csv 20 > gpurun_out/prof_$TAG/steady.txt
cat gpurun_out/traffic_$TAG/traffic_$TAG.json
head -8 gpurun_out/prof_$TAG/steady.txt
