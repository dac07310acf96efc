#!/bin/bash
# HBM traffic of the round kernels over the bench's timed region: FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md, HBM section), then
# tools/traffic_summary.py -> traffic_<tag>.json (copied to profiles/ as evidence).
# usage: tools/traffic.sh <nodes> <steps> <warmup> <tag>
set -u
PY=$(command -v python3)  # (an absolute path after rocprofv3's --: no PATH lookup in the profiled exec)
N=${1:-65536}; K=${2:-20}; W=${3:-20}; TAG=${4:-r01}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/traffic_$TAG
export TMPDIR=/tmp
ARGS="bench.py --nodes $N --steps $K --warmup $W --no-cpu-baseline --no-extras --no-traffic"
RE='k_phase[123]|k_p2_|k_lookup_keys'
timeout -k 10 600 rocprofv3 --kernel-include-regex "$RE" --pmc FETCH_SIZE -d gpurun_out/traffic_$TAG/fetch -o run --output-format csv -- "$PY" $ARGS > gpurun_out/traffic_$TAG/fetch.log 2>&1
rc=$?; echo "fetch exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-include-regex "$RE" --pmc WRITE_SIZE -d gpurun_out/traffic_$TAG/write -o run --output-format csv -- "$PY" $ARGS > gpurun_out/traffic_$TAG/write.log 2>&1
rc=$?; echo "write exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/traffic_summary.py gpurun_out/traffic_$TAG $K > gpurun_out/traffic_$TAG/traffic_$TAG.json
