#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md, rocprofv3 section).
# usage: tools/profile.sh <nodes> <steps> <warmup> <tag>
set -u
PY=$(command -v python3)  # (an absolute path after rocprofv3's --: no PATH lookup in the profiled exec)
N=${1:-65536}; K=${2:-5}; W=${3:-20}; TAG=${4:-r01}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
ARGS="bench.py --nodes $N --steps $K --warmup $W --no-cpu-baseline --no-extras --no-traffic"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- "$PY" $ARGS > gpurun_out/prof_$TAG/trace.log 2>&1
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
[ "${PROFILE_PMC:-1}" = 1 ] || exit 0
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$TAG/fetch -o run --output-format csv -- "$PY" $ARGS > gpurun_out/prof_$TAG/fetch.log 2>&1
rc=$?; echo "fetch exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$TAG/write -o run --output-format csv -- "$PY" $ARGS > gpurun_out/prof_$TAG/write.log 2>&1
rc=$?; echo "write exit $rc"; exit $rc
