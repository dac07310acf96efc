#!/bin/bash
# parity tests, then bench probes at growing sizes; stop at the first crash/timeout
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
for n in 4096 16384; do
  timeout -k 10 300 python bench.py --nodes $n --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err
  rc=$?; echo "bench $n exit $rc"; tail -c 1500 gpurun_out/bench_$n.json; tail -3 gpurun_out/bench_$n.err
  [ $rc -eq 0 ] || exit $rc
done
