#!/bin/bash
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_node.py > gpurun_out/pytest_r03g.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03g.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_kstats.sh default nopre head default || exit $?
AB_PMC=0 AB_MODE=bench bash tools/gpu_ab.sh default nopre head default nopre head
