#!/bin/bash
# parity tests (all GPU tests), headline bench, steady-state kernel trace, phase-2 diag
set -u
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
PROFILE_PMC=0 bash tools/profile.sh 65536 20 20 $TAG && python3 tools/trace_summary.py gpurun_out/prof_$TAG/trace/run_kernel_trace.csv 20 > gpurun_out/prof_$TAG/steady.txt; head -8 gpurun_out/prof_$TAG/steady.txt
[ "${DIAG:-1}" = 1 ] || exit 0
RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip_diag.so timeout -k 10 300 python -u tools/diag.py > gpurun_out/diag_$TAG.log 2>&1; tail -9 gpurun_out/diag_$TAG.log
