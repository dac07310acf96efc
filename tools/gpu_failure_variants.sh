#!/bin/bash
# config 5 (failure workload, 1 GPU) for each variant library given ("default"
# = the in-tree build): ms/round and kernel times.
set -u
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload failure --no-cpu-baseline > gpurun_out/fvar_$v.json 2> gpurun_out/fvar_$v.err || { echo "$v failed"; tail -3 gpurun_out/fvar_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/fvar_$v.json')); print('$v', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
