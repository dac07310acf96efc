#!/bin/bash
# Round 6 measurement pass on the final tree: the -m gpu suite, the default
# bench line (the driver's command), a rocprofv3 kernel-trace --stats profile
# of the headline, the JS drop-in ring benchmark and the ring update profile.
# usage: tools/gpu_r06_final.sh TAG [skip-tests]
set -u
TAG=$1
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
PY=$(command -v python3)
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
python3 -c "
import json; d = json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1])
print('ms/round', d['ms_per_step'], 'frac', d['roofline']['frac'], 'of_box', d['roofline'].get('frac_of_box'))
print('clk', d.get('clocks', {}).get('sclk_during_MHz'), 'box', {k: d['box_ceiling'][k] for k in ('stream16_GBps', 'rand16_rmw_per_s')})
print('c5', d.get('config5', {}).get('ms_per_step'), 'obs', d.get('observed_checksums', {}).get('checksums_ms'), 'c3', d.get('config3', {}).get('ms_per_step'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- "$PY" bench.py \
    --steps 20 --no-cpu-baseline --no-extras --no-traffic > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$TAG.log; exit $rc; }
python3 tools/trace_summary.py $(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1) 20 > gpurun_out/prof_$TAG.txt 2>&1
head -40 gpurun_out/prof_$TAG.txt
if command -v node > /dev/null; then
  timeout -k 10 300 node tools/js_ring_addremove.js gpu 5 > gpurun_out/js_ring_$TAG.json 2>&1 && cat gpurun_out/js_ring_$TAG.json
fi
timeout -k 10 300 python -u tools/ring_profile.py 3 > gpurun_out/ring_profile_$TAG.json 2>&1 && cat gpurun_out/ring_profile_$TAG.json
