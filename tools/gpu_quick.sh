#!/bin/bash
# parity tests, then the headline bench (no CPU baseline) and the RP_DIAG section split
set -u
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip_diag.so timeout -k 10 200 python -u tools/diag.py > gpurun_out/diag_$TAG.log 2>&1
rc=$?; cat gpurun_out/diag_$TAG.log; exit $rc
