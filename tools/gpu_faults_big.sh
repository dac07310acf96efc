#!/bin/bash
# GPU suite, then config 5 single-shard and on 4 in-process shards (one GPU)
set -u
TAG=${1:-f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload failure > gpurun_out/failure_$TAG.json 2> gpurun_out/failure_$TAG.err
rc=$?; echo "failure exit $rc"; cat gpurun_out/failure_$TAG.json; tail -3 gpurun_out/failure_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload failure --shards 4 > gpurun_out/failure4_$TAG.json 2> gpurun_out/failure4_$TAG.err
rc=$?; echo "failure shards4 exit $rc"; cat gpurun_out/failure4_$TAG.json; tail -3 gpurun_out/failure4_$TAG.err; exit $rc
