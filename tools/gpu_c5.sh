#!/bin/bash
# GPU tests, then config 5 (single shard), then the headline bench (no CPU baseline)
set -u
TAG=${1:-c5}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload failure > gpurun_out/failure_$TAG.json 2> gpurun_out/failure_$TAG.err
rc=$?; echo "failure exit $rc"; cat gpurun_out/failure_$TAG.json; tail -2 gpurun_out/failure_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; exit $rc
