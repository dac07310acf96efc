#!/bin/bash
# PMC passes over the config-4 round kernels (one counter group per
# rocprofv3 run), summarised per kernel: where the issue and merge kernels'
# wave cycles go (active VALU / VMEM / LDS / SALU vs parked), instruction mix,
# L2 hit rate.  usage: tools/gpu_pmc_round.sh <tag>
set -u
TAG=${1:-r03}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export PMC_RE='k_phase1|k_p2_respond|k_p2_apply|k_phase3'
export PMC_PASSES="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM|TCC_HIT_sum TCC_MISS_sum|FETCH_SIZE|WRITE_SIZE"
bash tools/pmc.sh 65536 3 20 $TAG || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG 3 > gpurun_out/pmc_$TAG/summary.txt
cat gpurun_out/pmc_$TAG/summary.txt
