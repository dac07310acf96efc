#!/bin/bash
# config-5 per-round counters (1 and 4 shards) + lookup directory / keys-per-thread A/B
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_c5.py 32768 1 > gpurun_out/probe_c5_sh1.txt 2>&1 || { echo probe1 failed; tail -3 gpurun_out/probe_c5_sh1.txt; exit 1; }
timeout -k 10 400 python -u tools/probe_c5.py 32768 4 > gpurun_out/probe_c5_sh4.txt 2>&1 || { echo probe4 failed; tail -3 gpurun_out/probe_c5_sh4.txt; exit 1; }
for G in 4 1; do
  timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl_sh$G -o run -- python3 tools/probe_c5.py 32768 $G > gpurun_out/tl_sh$G.log 2>&1 || { echo trace $G failed; tail -3 gpurun_out/tl_sh$G.log; exit 1; }
  K=$(find gpurun_out/tl_sh$G -name "run_kernel_trace.csv" | head -1); M=$(find gpurun_out/tl_sh$G -name "run_memory_copy_trace.csv" | head -1)
  echo "== timeline shards=$G"; python3 tools/timeline.py $K $M --skip 0.3 | tee gpurun_out/timeline_sh$G.txt
done
for v in default d22 d23 kpt2 kpt4 default d22 d23 kpt2 kpt4; do
  if [ $v = default ]; then export RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip.so; else export RINGPOP_HIP_LIB=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload lookup --no-cpu-baseline > gpurun_out/lk_$v.json 2> gpurun_out/lk_$v.err || { echo lk $v failed; tail -3 gpurun_out/lk_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/lk_$v.json')); print('lookup $v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('parity'))"
done
