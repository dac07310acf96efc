#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over a
# short bench.py run; restricted to the round kernels by regex.
# usage: tools/pmc_lookup.sh 0 0 0 <tag>  (config-3 lookup kernel)
set -u
PY=$(command -v python3)  # (an absolute path after rocprofv3's --: no PATH lookup in the profiled exec)
N=${1:-65536}; K=${2:-3}; W=${3:-20}; TAG=${4:-r01}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
ARGS="bench.py --workload lookup --steps 3 --warmup 3 --no-cpu-baseline"
RE=k_lookup_keys
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-include-regex "$RE" --pmc $P -d gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- "$PY" $ARGS > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i ($P) exit $rc"; [ $rc -eq 0 ] || exit $rc
done
