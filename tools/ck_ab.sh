#!/bin/bash
# A/B of the many-view checksum kernels on one GPU box: first the checksum
# parity tests (lane-per-view fixtures, both paths at full size) with the
# in-tree library, then all 65,536 checksums of config 4 through the lane path
# (tools/ck_paths.py, 3 reads after 20 rounds) per library variant, in the
# order given ("default" = the in-tree library, NAME = a
# tools/build_variant.sh build in ringpop_amd/variants/).
# usage: CK_VARIANTS="default NAME default NAME" bash tools/ck_ab.sh
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread -m gpu -k "checksum or lane" > gpurun_out/pytest_ck.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ck.log; [ $rc -eq 0 ] || exit $rc
for v in ${CK_VARIANTS:-default}; do
  if [ $v = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  CK_MODES=lanes RINGPOP_HIP_LIB=$L timeout -k 10 300 python -u tools/ck_paths.py 65536 20 3 > gpurun_out/ck_$v.json 2>/dev/null || exit $?
  echo $v $(cat gpurun_out/ck_$v.json)
done
