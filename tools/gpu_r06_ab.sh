#!/bin/bash
# Round 6 A/B pass: the -m gpu suite on the in-tree library, then interleaved
# per-kernel rocprof stats of the named variants, then one PMC instruction
# pass (SQ_INSTS_*) over the issue and merge kernels per variant.
# usage: tools/gpu_r06_ab.sh TAG [--no-tests] variant ...
set -u
TAG=$1; shift
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${1:-}" = --no-tests ]; then shift; else
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
bash tools/gpu_kstats.sh "$@" > gpurun_out/kstats_$TAG.txt 2>&1 || { cat gpurun_out/kstats_$TAG.txt; exit 1; }
cat gpurun_out/kstats_$TAG.txt
timeout -k 10 300 python -u tools/ring_profile.py 3 > gpurun_out/ring_profile_$TAG.json 2>&1 && cat gpurun_out/ring_profile_$TAG.json || { echo "ring profile failed"; tail -5 gpurun_out/ring_profile_$TAG.json; exit 1; }
seen=""
for v in "$@"; do
  case " $seen " in *" $v "*) continue ;; esac; seen="$seen $v"
  if [ "$v" = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L PMC_RE='k_phase1|k_p2_respond|k_phase3|k_p2_apply' \
  PMC_PASSES='SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_ACTIVE_INST_VALU' \
    bash tools/pmc.sh 65536 3 20 insts_${TAG}_$v > /dev/null || { echo "pmc $v failed"; exit 1; }
  echo "== pmc $v"; python3 tools/pmc_summary.py gpurun_out/pmc_insts_${TAG}_$v 3 | tee gpurun_out/pmc_insts_${TAG}_$v.txt | grep -A9 "k_phase1\|k_p2_respond" | grep "k_\|VALU\|SALU"
done
