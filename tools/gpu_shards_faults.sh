#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_shards.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_shards.log | head -40; tail -30 gpurun_out/pytest_shards.log; exit $rc
