#!/bin/bash
# PMC passes over k_checksums_pc: one read of all 65,536 checksums of
# config 4 (tools/ck_paths.py, lane path), one counter group per rocprofv3
# run, kernel trace only; summary per dispatch:
#   python3 tools/pmc_summary.py gpurun_out/pmc_ck_<tag> 1
# usage: tools/pmc_ck.sh <tag>
set -u
PY=$(command -v python3)  # (an absolute path after rocprofv3's --)
TAG=${1:-ck}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/pmc_ck_$TAG
export TMPDIR=/tmp
PASSES=${PMC_PASSES:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM"}
i=0
IFS='|' read -r -a GROUPS_ <<< "$PASSES"
for P in "${GROUPS_[@]}"; do
  i=$((i+1))
  CK_MODES=lanes timeout -k 10 300 rocprofv3 --kernel-include-regex k_checksums_pc --pmc $P -d gpurun_out/pmc_ck_$TAG/p$i -o run --output-format csv -- "$PY" tools/ck_paths.py 65536 20 1 > gpurun_out/pmc_ck_$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i ($P) exit $rc"; [ $rc -eq 0 ] || exit $rc
done
