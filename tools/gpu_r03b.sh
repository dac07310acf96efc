#!/bin/bash
# round-3 checks: the new parity tests, then config 5 at 65,536 nodes on 4 in-process shards
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s -m gpu tests/test_gpu_parity.py -k "compaction or views_argument" tests/test_gpu_node.py tests/test_js.py tests/test_gpu_rccl.py tests/test_capi.py > gpurun_out/pytest_r03b.log 2>&1
rc=$?; echo pytest $rc; grep -E "compactions|passed|failed|PASS|FAIL|SKIP|Error" gpurun_out/pytest_r03b.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -s -m gpu tests/test_gpu_fullsize.py -k "invariants" > gpurun_out/pytest_r03b_full.log 2>&1
rc=$?; echo full $rc; grep -E "compactions|passed|failed" gpurun_out/pytest_r03b_full.log | tail
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/f64_sh4_r03b.json 2> gpurun_out/f64_sh4_r03b.err
rc=$?; echo f64sh4 $rc; cat gpurun_out/f64_sh4_r03b.json; tail -3 gpurun_out/f64_sh4_r03b.err
