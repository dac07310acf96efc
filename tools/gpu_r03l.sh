#!/bin/bash
# straight-line issue pass 1 + host worker thread per in-process shard:
# parity (sim, shard and node tests), kstats A/B against the HEAD build,
# config 5 at 32,768 nodes and config 4 on 4 in-process shards with and
# without shard threads, then per-round host/GPU traces (tools/round_gaps.py)
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $P tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_node.py > gpurun_out/pytest_r03l.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03l.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_kstats.sh default base default base || exit 1
for t in 1 0 1 0; do
  RP_SHARD_THREADS=$t timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --shards 4 --no-cpu-baseline > gpurun_out/f32_sh4_t$t.json 2> gpurun_out/f32_sh4_t$t.err || { echo f32 t$t failed; tail -3 gpurun_out/f32_sh4_t$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f32_sh4_t$t.json')); print('c5 32k/4 threads=$t', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'])"
  RP_SHARD_THREADS=$t timeout -k 10 300 python -u bench.py --shards 4 --no-extras --no-cpu-baseline > gpurun_out/c4_sh4_t$t.json 2> gpurun_out/c4_sh4_t$t.err || { echo c4 t$t failed; tail -3 gpurun_out/c4_sh4_t$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4_sh4_t$t.json')); print('c4 sh4 threads=$t', d['ms_per_step'], d['kernel_ms'])"
done
timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --no-cpu-baseline > gpurun_out/f32_sh1.json 2> gpurun_out/f32_sh1.err || { echo f32 sh1 failed; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/f32_sh1.json')); print('c5 32k/1', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'])"
for s in 1 4; do
  timeout -s KILL 400 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/rg_sh$s -o run -- python3 tools/probe_c5.py 32768 $s > gpurun_out/rg_sh$s.log 2>&1 || { echo trace $s failed; tail -3 gpurun_out/rg_sh$s.log; exit 1; }
  python3 tools/round_gaps.py gpurun_out/rg_sh$s k_seen_clear $s --from 46 --to 58 > gpurun_out/round_gaps_sh$s.txt
  python3 tools/round_gaps.py gpurun_out/rg_sh$s k_seen_clear $s --from 30 --to 40 > gpurun_out/round_gaps_mid_sh$s.txt
  head -20 gpurun_out/round_gaps_sh$s.txt
  find gpurun_out/rg_sh$s -name "*.csv" -size +20M -delete
done
