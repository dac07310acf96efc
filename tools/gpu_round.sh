#!/bin/bash
# one GPU session: parity tests + smoke, headline bench, rocprofv3 kernel-trace stats.
# stops at the first failure without starting more GPU work.
# usage: tools/gpu_round.sh <tag>
set -u
TAG=${1:-r01}
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
PROFILE_PMC=${PROFILE_PMC:-0} bash tools/profile.sh 65536 5 20 $TAG
