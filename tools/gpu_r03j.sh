#!/bin/bash
# batched in-process copies + parallel slot planning: shard parity, then config-5 benches 1 vs 4 shards
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
timeout -k 10 600 $P tests/test_gpu_shards.py tests/test_gpu_parity.py > gpurun_out/pytest_r03j.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03j.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $P tests/test_gpu_fullsize.py -k "shards" > gpurun_out/pytest_r03j_full.log 2>&1
rc=$?; echo full $rc; tail -2 gpurun_out/pytest_r03j_full.log
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl2_sh4 -o run -- python3 tools/probe_c5.py 32768 4 > gpurun_out/tl2_sh4.log 2>&1 || { echo trace failed; tail -3 gpurun_out/tl2_sh4.log; exit 1; }
K=$(find gpurun_out/tl2_sh4 -name "run_kernel_trace.csv" | head -1); M=$(find gpurun_out/tl2_sh4 -name "run_memory_copy_trace.csv" | head -1)
python3 tools/timeline.py $K $M --skip 0.3 > gpurun_out/timeline2_sh4.txt; head -40 gpurun_out/timeline2_sh4.txt
for s in 1 4; do
  timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --shards $s --no-cpu-baseline > gpurun_out/f32_sh$s.json 2> gpurun_out/f32_sh$s.err || { echo f32 $s failed; tail -3 gpurun_out/f32_sh$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f32_sh$s.json')); print('32k/$s', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'], (d.get('exchange') or {}).get('bytes_per_round_rank0'))"
done
timeout -k 10 400 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/f64_sh4.json 2> gpurun_out/f64_sh4.err || { echo f64 failed; tail -3 gpurun_out/f64_sh4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/f64_sh4.json')); print('64k/4', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'], (d.get('exchange') or {}).get('bytes_per_round_rank0'))"
