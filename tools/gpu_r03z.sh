#!/bin/bash
# loopback rank transport: the rank path vs in-process shards, then the shard parity tests
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_loop_ranks.py > gpurun_out/pytest_r03z_loop.log 2>&1
rc=$?; echo loop $rc; tail -8 gpurun_out/pytest_r03z_loop.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_shards.py tests/test_gpu_parity.py > gpurun_out/pytest_r03z.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03z.log
