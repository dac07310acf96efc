#!/bin/bash
# fewer host calls per sharded round (batched resets, merged collective
# scopes, small shuffle grid, shard threads): parity, then config 5 / config 4
# on 4 in-process shards against the HEAD build, interleaved; config 5 at
# 65,536 nodes on 4 shards; the headline bench
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
true


lib_of() { if [ "$1" = default ]; then echo "$PWD/ringpop_amd/libringpop_hip.so"; else echo "$PWD/ringpop_amd/variants/libringpop_hip_$1.so"; fi; }
for v in default base default base; do
  L=$(lib_of $v)
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --shards 4 --no-cpu-baseline > gpurun_out/m_f32_$v.json 2> gpurun_out/m_f32_$v.err || { echo f32 $v failed; tail -3 gpurun_out/m_f32_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/m_f32_$v.json')); x=d.get('exchange') or {}; print('c5 32k/4 $v', d['ms_per_step'], d.get('first_agreement_round'), x.get('bytes_per_round_rank0'), x.get('bytes_per_round_max_rank'))"
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --shards 4 --no-extras --no-cpu-baseline > gpurun_out/m_c4_$v.json 2> gpurun_out/m_c4_$v.err || { echo c4 $v failed; tail -3 gpurun_out/m_c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/m_c4_$v.json')); x=d.get('exchange') or {}; print('c4 sh4 $v', d['ms_per_step'], x.get('bytes_per_round_rank0'))"
done
timeout -k 10 300 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/m_f64_sh4.json 2> gpurun_out/m_f64_sh4.err || { echo f64 failed; tail -3 gpurun_out/m_f64_sh4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/m_f64_sh4.json')); x=d.get('exchange') or {}; print('c5 64k/4', d['ms_per_step'], d.get('first_agreement_round'), x.get('bytes_per_round_rank0'), x.get('bytes_per_round_max_rank'), d['end_state'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/m_c4.json 2> gpurun_out/m_c4.err || { echo c4 failed; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/m_c4.json')); print('c4 1 GPU', d['ms_per_step'], d['roofline']['frac'])"
