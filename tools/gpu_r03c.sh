#!/bin/bash
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread -s -m gpu tests/test_gpu_fullsize.py -k "config5" > gpurun_out/pytest_r03c_full.log 2>&1
rc=$?; echo full $rc; grep -E "passed|failed|Error|assert" gpurun_out/pytest_r03c_full.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err || { tail -3 gpurun_out/bench_r03c.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r03c.json')); print(d['ms_per_step'], d['kernel_ms']); print(json.dumps(d['stages'], indent=0)[:3000])"
bash tools/gpu_pmc_round.sh r03c
