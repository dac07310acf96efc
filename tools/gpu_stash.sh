#!/bin/bash
# parity with the default build, parity with a 16-entry stash (overflow path), then A/B vs the old build
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
RINGPOP_HIP_LIB=$PWD/ringpop_amd/variants/libringpop_hip_st16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_st16.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_st16.log; [ $rc -eq 0 ] || exit $rc
bash tools/alt_ab.sh
