#!/bin/bash
# identical-view issue filter: parity (incl. full size), config-5 probe, config-5 benches
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
timeout -k 10 600 $P tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_node.py > gpurun_out/pytest_r03i.log 2>&1
rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_r03i.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $P -s tests/test_gpu_fullsize.py > gpurun_out/pytest_r03i_full.log 2>&1
rc=$?; echo full $rc; grep -E "compactions|passed|failed" gpurun_out/pytest_r03i_full.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_c5.py 32768 1 > gpurun_out/probe_c5_sh1_sv.txt 2>&1 || { echo probe1 failed; exit 1; }
timeout -k 10 400 python -u tools/probe_c5.py 32768 4 > gpurun_out/probe_c5_sh4_sv.txt 2>&1 || { echo probe4 failed; exit 1; }
grep total gpurun_out/probe_c5_sh1_sv.txt
timeout -k 10 400 python -u bench.py --workload failure --no-cpu-baseline > gpurun_out/bench_failure_sv.json 2> gpurun_out/bench_failure_sv.err || { echo bench failure failed; tail -3 gpurun_out/bench_failure_sv.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_failure_sv.json')); print('failure', d['ms_per_step'], d.get('first_agreement_round'), d['kernel_ms'])"
