#!/bin/bash
# sharded-simulation parity tests, then exchange volumes at full size (1 vs 4 in-process shards)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_shards.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -12 gpurun_out/pytest_shards.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/exchange_diag.py 65536 4 > gpurun_out/xdiag.log 2>&1
rc=$?; echo "xdiag exit $rc"; cat gpurun_out/xdiag.log; exit $rc
