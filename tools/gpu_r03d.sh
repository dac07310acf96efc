#!/bin/bash
# prefix packing + 16-bit lookup directory: parity, then A/B timings
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_node.py tests/test_gpu_wire.py > gpurun_out/pytest_r03d.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03d.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $P -s tests/test_gpu_fullsize.py -k "not config5_full_size_shards" > gpurun_out/pytest_r03d_full.log 2>&1
rc=$?; echo full $rc; grep -E "compactions|passed|failed" gpurun_out/pytest_r03d_full.log | tail -4
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_kstats.sh default noprefix default noprefix || exit $?
for v in default dir32 dir16b21; do
  if [ $v = default ]; then export RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip.so; else export RINGPOP_HIP_LIB=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload lookup --no-cpu-baseline > gpurun_out/lk_$v.json 2> gpurun_out/lk_$v.err || { echo lk $v failed; tail -3 gpurun_out/lk_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/lk_$v.json')); print('lookup $v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('parity'))"
done
