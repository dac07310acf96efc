#!/bin/bash
# config 3 lookup: non-temporal streams (default) vs HEAD (base) vs a 2^22-bucket 16-bit directory (d22), interleaved
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
lib_of() { if [ "$1" = default ]; then echo "$PWD/ringpop_amd/libringpop_hip.so"; else echo "$PWD/ringpop_amd/variants/libringpop_hip_$1.so"; fi; }
for v in default base d22 default base d22; do
  RINGPOP_HIP_LIB=$(lib_of $v) timeout -k 10 300 python -u bench.py --workload lookup --no-cpu-baseline > gpurun_out/v_lk_$v.json 2> gpurun_out/v_lk_$v.err || { echo lookup $v failed; tail -3 gpurun_out/v_lk_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/v_lk_$v.json')); print('lookup $v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('parity'))"
done
