#!/bin/bash
# Host-idle time per round of the rank path: kernel, HIP runtime API and copy
# traces of `bench.py --loop-ranks G` (config 4, G rank threads on one GPU,
# the one-process-per-GPU code with a loopback transport), split per round by
# tools/round_gaps.py over the timed rounds.  (No --pmc in this run.)
# usage: tools/gpu_gaps.sh tag [G] [nodes] [steps]
set -u
TAG=$1; G=${2:-8}; N=${3:-65536}; K=${4:-10}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
PY=$(command -v python3)  # (an absolute path after rocprofv3's --)
PRE=20; W=3
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d gpurun_out/gaps_$TAG -o run \
    --output-format csv -- "$PY" bench.py --loop-ranks $G --nodes $N --steps $K --warmup $W --preroll $PRE \
    --no-cpu-baseline --no-extras --no-traffic > gpurun_out/gaps_$TAG.log 2>&1
rc=$?; echo "rocprofv3 exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/gaps_$TAG.log; exit $rc; }
python3 tools/round_gaps.py gpurun_out/gaps_$TAG k_round_start $G --from $((PRE + W + 1)) > gpurun_out/gaps_$TAG.txt
rc=$?; grep -E "mean over|hipStreamSynchronize|hipMemcpy" gpurun_out/gaps_$TAG.txt; exit $rc
