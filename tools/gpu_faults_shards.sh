#!/bin/bash
# sharded fault tests, then config 5 on 4 in-process shards (one GPU)
set -u
TAG=${1:-f}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_shards.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_shards.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload failure --shards 4 > gpurun_out/failure4_$TAG.json 2> gpurun_out/failure4_$TAG.err
rc=$?; echo "failure shards4 exit $rc"; cat gpurun_out/failure4_$TAG.json; tail -3 gpurun_out/failure4_$TAG.err; exit $rc
