#!/bin/bash
# GPU parity with the default build, then headline bench per variant (twice)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh "$@" && bash tools/gpu_variants.sh "$@"
