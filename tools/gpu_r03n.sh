#!/bin/bash
# config 5 at 65,536 nodes on 4 in-process shards: shard threads off / on, interleaved
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for t in 0 1 0 1; do
  RP_SHARD_THREADS=$t timeout -k 10 300 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/n_f64_t$t.json 2> gpurun_out/n_f64_t$t.err || { echo f64 t$t failed; tail -3 gpurun_out/n_f64_t$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/n_f64_t$t.json')); x=d.get('exchange') or {}; print('c5 64k/4 threads=$t', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'])"
done
