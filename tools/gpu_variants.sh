#!/bin/bash
# headline bench for each ringpop_amd/variants/libringpop_hip_<name>.so given as
# arguments, in the order given ("default" = the in-tree build; repeat names
# to interleave A/B runs on one box)
set -u
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err
  rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var_$v.json')); print('$v', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])" || { echo "$v failed rc=$rc"; tail -3 gpurun_out/var_$v.err; exit 1; }
done
