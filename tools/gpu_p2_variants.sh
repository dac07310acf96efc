#!/bin/bash
# k_phase2 variants: headline ms/round and the kernel's FETCH/WRITE bytes per
# variant library (ringpop_amd/variants/libringpop_hip_<name>.so; "default" =
# the in-tree build).  usage: tools/gpu_p2_variants.sh name ...
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  export RINGPOP_HIP_LIB=$L
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "$v bench failed"; tail -3 gpurun_out/var_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/var_$v.json')); print('$v', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  PMC_RE='k_phase2' PMC_PASSES='FETCH_SIZE|WRITE_SIZE' bash tools/pmc.sh 65536 3 20 var_$v > /dev/null || { echo "$v pmc failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/pmc_var_$v 2 | grep -E "k_phase2|FETCH|WRITE"
done
