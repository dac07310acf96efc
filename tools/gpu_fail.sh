#!/bin/bash
# parity tests, config 3 lookup bench, then the config 5 mass-failure run
set -u
TAG=${1:-r01}
bash tools/gpu_check.sh || exit $?
timeout -k 10 400 python -u bench.py --workload lookup --steps 10 --warmup 3 > gpurun_out/lookup_$TAG.json 2> gpurun_out/lookup_$TAG.err
rc=$?; echo "lookup exit $rc"; cat gpurun_out/lookup_$TAG.json; tail -5 gpurun_out/lookup_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload failure > gpurun_out/failure_$TAG.json 2> gpurun_out/failure_$TAG.err
rc=$?; echo "failure exit $rc"; cat gpurun_out/failure_$TAG.json; tail -5 gpurun_out/failure_$TAG.err; exit $rc
