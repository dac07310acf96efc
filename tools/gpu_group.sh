#!/bin/bash
# grouping (handleOrProxyAll) parity tests, then the config-3 lookup bench line
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "group" > gpurun_out/pytest_group.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_group.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload lookup > gpurun_out/bench_lookup.json 2> gpurun_out/bench_lookup.err
rc=$?; cat gpurun_out/bench_lookup.json; tail -5 gpurun_out/bench_lookup.err; exit $rc
