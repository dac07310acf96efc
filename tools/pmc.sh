#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over a
# short bench.py run; restricted to the round kernels by regex.
# usage: tools/pmc.sh <nodes> <steps> <warmup> <tag>
set -u
PY=$(command -v python3)  # (an absolute path after rocprofv3's --: no PATH lookup in the profiled exec)
N=${1:-65536}; K=${2:-3}; W=${3:-20}; TAG=${4:-r01}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
ARGS="bench.py --nodes $N --steps $K --warmup $W --no-cpu-baseline --no-extras --no-traffic"
RE=${PMC_RE:-'k_phase[123]'}
# PMC_PASSES: counter groups separated by '|' (default: all five groups)
PASSES=${PMC_PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA|TCC_HIT_sum TCC_MISS_sum|SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"}
i=0
IFS='|' read -r -a GROUPS_ <<< "$PASSES"
for P in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-include-regex "$RE" --pmc $P -d gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- "$PY" $ARGS > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i ($P) exit $rc"; [ $rc -eq 0 ] || exit $rc
done
