#!/bin/bash
# iterator over pingable bits: parity, config 5 A/B (1 and 4 shards), per-round probes
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_node.py tests/test_gpu_wire.py > gpurun_out/pytest_r03x.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03x.log
[ $rc -eq 0 ] || exit $rc
lib_of() { if [ "$1" = default ]; then echo "$PWD/ringpop_amd/libringpop_hip.so"; else echo "$PWD/ringpop_amd/variants/libringpop_hip_$1.so"; fi; }
for v in default base default base; do
  L=$(lib_of $v)
  RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload failure --no-cpu-baseline > gpurun_out/x_f64_$v.json 2> gpurun_out/x_f64_$v.err || { echo f64 $v failed; tail -3 gpurun_out/x_f64_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/x_f64_$v.json')); print('c5 64k/1 $v', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'])"
done
RINGPOP_HIP_LIB=$(lib_of default) timeout -k 10 300 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/x_f64s4.json 2> gpurun_out/x_f64s4.err || { echo f64s4 failed; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/x_f64s4.json')); x=d.get('exchange') or {}; print('c5 64k/4', d['ms_per_step'], d.get('first_agreement_round'), x.get('bytes_per_round_max_rank'))"
timeout -k 10 300 python3 -u tools/probe_c5.py 65536 1 > gpurun_out/probe64_sh1.log 2>&1 || { echo probe1 failed; exit 1; }
timeout -k 10 300 python3 -u tools/probe_c5.py 65536 4 > gpurun_out/probe64_sh4.log 2>&1 || { echo probe4 failed; exit 1; }
paste -d' ' <(awk '{print $1, $2, $4, $5}' gpurun_out/probe64_sh1.log) <(awk '{print $2, $4, $5}' gpurun_out/probe64_sh4.log) | head -62
