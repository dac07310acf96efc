#!/bin/bash
# exchange buffers presized for fault runs: shard parity, growth log, config 5 on 4 shards at 65,536 / 32,768 nodes
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_gpu_shards.py tests/test_gpu_parity.py > gpurun_out/pytest_r03u.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03u.log
[ $rc -eq 0 ] || exit $rc
RP_DEBUG_GROW=1 timeout -k 10 300 python3 -u tools/probe_c5.py 65536 4 > gpurun_out/grow64b.log 2>&1 || { echo probe failed; tail -3 gpurun_out/grow64b.log; exit 1; }
grep -c grow gpurun_out/grow64b.log; grep grow gpurun_out/grow64b.log | awk '{t+=$(NF-1)} END {print "total grow ms", t}'; grep "^1[0-2] " gpurun_out/grow64b.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/u_f64s4_$i.json 2> gpurun_out/u_f64s4_$i.err || { echo f64s4 failed; tail -3 gpurun_out/u_f64s4_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/u_f64s4_$i.json')); x=d.get('exchange') or {}; print('c5 64k/4', d['ms_per_step'], d.get('first_agreement_round'), x.get('bytes_per_round_max_rank'), d.get('device_memory_used_gb'), d['end_state']['every_failed_faulty'])"
  timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --shards 4 --no-cpu-baseline > gpurun_out/u_f32s4_$i.json 2> gpurun_out/u_f32s4_$i.err || { echo f32s4 failed; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/u_f32s4_$i.json')); x=d.get('exchange') or {}; print('c5 32k/4', d['ms_per_step'], d.get('first_agreement_round'), x.get('bytes_per_round_max_rank'))"
done
