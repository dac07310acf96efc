#!/bin/bash
# config 3 lookup bench, merge-kernel HBM traffic passes, config 5 failure run
set -u
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload lookup --steps 10 --warmup 3 > gpurun_out/lookup_$TAG.json 2> gpurun_out/lookup_$TAG.err
rc=$?; echo "lookup exit $rc"; cat gpurun_out/lookup_$TAG.json; tail -5 gpurun_out/lookup_$TAG.err; [ $rc -eq 0 ] || exit $rc
bash tools/traffic.sh 65536 20 20 $TAG; rc=$?; echo "traffic exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload failure > gpurun_out/failure_$TAG.json 2> gpurun_out/failure_$TAG.err
rc=$?; echo "failure exit $rc"; cat gpurun_out/failure_$TAG.json; tail -5 gpurun_out/failure_$TAG.err; exit $rc
