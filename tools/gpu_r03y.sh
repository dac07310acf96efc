#!/bin/bash
# current (reasserted) bits: parity incl. full-size config 5 on 1 and 4 shards, then config 5 A/B
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_node.py tests/test_gpu_wire.py tests/test_gpu_fullsize.py > gpurun_out/pytest_r03y.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03y.log
[ $rc -eq 0 ] || exit $rc
lib_of() { if [ "$1" = default ]; then echo "$PWD/ringpop_amd/libringpop_hip.so"; else echo "$PWD/ringpop_amd/variants/libringpop_hip_$1.so"; fi; }
for v in default base default base; do
  L=$(lib_of $v)
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload failure --no-cpu-baseline > gpurun_out/y_f64_$v.json 2> gpurun_out/y_f64_$v.err || { echo f64 $v failed; tail -3 gpurun_out/y_f64_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/y_f64_$v.json')); print('c5 64k/1 $v', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'])"
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/y_f64s4_$v.json 2> gpurun_out/y_f64s4_$v.err || { echo f64s4 $v failed; tail -3 gpurun_out/y_f64s4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/y_f64s4_$v.json')); x=d.get('exchange') or {}; print('c5 64k/4 $v', d['ms_per_step'], d.get('first_agreement_round'), x.get('bytes_per_round_max_rank'))"
done
for v in default base; do
  L=$(lib_of $v)
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --no-cpu-baseline > gpurun_out/y_f32_$v.json 2> gpurun_out/y_f32_$v.err || { echo f32 $v failed; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/y_f32_$v.json')); print('c5 32k/1 $v', d['ms_per_step'], d.get('first_agreement_round'))"
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --shards 4 --no-cpu-baseline > gpurun_out/y_f32s4_$v.json 2> gpurun_out/y_f32s4_$v.err || { echo f32s4 $v failed; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/y_f32s4_$v.json')); x=d.get('exchange') or {}; print('c5 32k/4 $v', d['ms_per_step'], d.get('first_agreement_round'), x.get('bytes_per_round_max_rank'))"
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/y_c4_$v.json 2> gpurun_out/y_c4_$v.err || { echo c4 $v failed; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/y_c4_$v.json')); print('c4 $v', d['ms_per_step'])"
done
