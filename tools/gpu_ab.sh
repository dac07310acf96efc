#!/bin/bash
# diag breakdown of phase 2, then headline bench per variant
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip_diag.so timeout -k 10 200 python -u tools/diag.py > gpurun_out/diag.log 2>&1
rc=$?; cat gpurun_out/diag.log | tail -12; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh "$@"
