#!/bin/bash
# round-3 checks: parity of the new paths (16-byte escapes + origin all-gather,
# shard streams), then sharded timings: config 4 and config 5 on 4 in-process
# shards (shard streams vs one stream), config 5 at 65,536 on 4 shards
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread -s -m gpu"
timeout -k 10 900 $P tests/test_gpu_node.py tests/test_js.py tests/test_gpu_rccl.py tests/test_capi.py tests/test_gpu_shards.py tests/test_gpu_wire.py > gpurun_out/pytest_r03b.log 2>&1
rc=$?; echo pytest $rc; grep -E "passed|failed|FAIL|Error" gpurun_out/pytest_r03b.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $P tests/test_gpu_parity.py > gpurun_out/pytest_r03b_par.log 2>&1
rc=$?; echo parity $rc; grep -E "passed|failed|FAIL|Error" gpurun_out/pytest_r03b_par.log | tail -12
[ $rc -eq 0 ] || exit $rc
for v in default onestream; do
  if [ $v = default ]; then export RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip.so; else export RINGPOP_HIP_LIB=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  timeout -k 10 300 python -u bench.py --shards 4 --no-extras --no-cpu-baseline > gpurun_out/c4_sh4_$v.json 2> gpurun_out/c4_sh4_$v.err || { echo c4 $v failed; tail -3 gpurun_out/c4_sh4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4_sh4_$v.json')); print('c4sh4 $v', d['ms_per_step'], d['kernel_ms'], d.get('exchange',{}).get('bytes_per_round_rank0'))"
  for s in 1 4; do
    timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --shards $s --no-cpu-baseline > gpurun_out/f32_sh${s}_$v.json 2> gpurun_out/f32_sh${s}_$v.err || { echo f32 $v $s failed; tail -3 gpurun_out/f32_sh${s}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/f32_sh${s}_$v.json')); print('f32 sh$s $v', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('exchange',{}).get('bytes_per_round_rank0'), d['device_memory_used_gb'])"
  done
done
unset RINGPOP_HIP_LIB
timeout -k 10 600 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/f64_sh4_r03b.json 2> gpurun_out/f64_sh4_r03b.err
rc=$?; echo f64sh4 $rc; cat gpurun_out/f64_sh4_r03b.json; tail -3 gpurun_out/f64_sh4_r03b.err
