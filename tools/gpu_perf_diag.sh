#!/bin/bash
# Where the round's time goes: the RP_DIAG build's cycle breakdown of k_phase2
# (tools/diag.py), PMC passes over the phase kernels (tools/pmc.sh), and the
# headline on 4 in-process shards (exchange volume per round).
# usage: tools/gpu_perf_diag.sh <tag>
set -u
TAG=${1:-r02}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip_diag.so timeout -k 10 200 python -u tools/diag.py > gpurun_out/diag_$TAG.json 2>&1
rc=$?; echo "diag exit $rc"; cat gpurun_out/diag_$TAG.json; [ $rc -eq 0 ] || exit $rc
bash tools/pmc.sh 65536 3 20 $TAG || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG 3 > gpurun_out/pmc_$TAG/summary.txt; cat gpurun_out/pmc_$TAG/summary.txt
timeout -k 10 400 python -u bench.py --shards 4 --no-extras --no-cpu-baseline --steps 10 > gpurun_out/bench_shards4_$TAG.json 2> gpurun_out/bench_shards4_$TAG.err
rc=$?; echo "shards4 exit $rc"; cat gpurun_out/bench_shards4_$TAG.json; tail -3 gpurun_out/bench_shards4_$TAG.err
