#!/bin/bash
# Config 4 on 4 in-process shards per variant library ("default" = in-tree):
# ms/round, exchange bytes/round.  usage: tools/gpu_shard_variants.sh name ...
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --shards ${SHARDS:-4} --no-extras --no-cpu-baseline > gpurun_out/shv_$v.json 2> gpurun_out/shv_$v.err || { echo "$v failed"; tail -3 gpurun_out/shv_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/shv_$v.json')); print('$v', d['ms_per_step'], d['kernel_ms'], d['exchange']['bytes_per_round_rank0'])"
done
