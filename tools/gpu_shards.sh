#!/bin/bash
# sharded-simulation parity tests, headline bench, 2-shard in-process bench at full size
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_shards.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -12 gpurun_out/pytest_shards.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_single.json 2> gpurun_out/bench_single.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_single.json; tail -3 gpurun_out/bench_single.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --no-cpu-baseline --shards 2 --steps 10 --warmup 10 > gpurun_out/bench_shards2.json 2> gpurun_out/bench_shards2.err
rc=$?; echo "bench shards exit $rc"; cat gpurun_out/bench_shards2.json; tail -3 gpurun_out/bench_shards2.err; exit $rc
