#!/bin/bash
# Round-6 GPU pass: the -m gpu suite, the default bench line (box ceilings,
# clocks), and one PMC instruction pass over the issue and merge kernels.
# usage: tools/gpu_r06_suite.sh TAG [skip-tests]
set -u
TAG=${1:-r06}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
python3 -c "
import json; d = json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1])
print('ms/round', d['ms_per_step'], 'frac', d['roofline']['frac'], 'box', d.get('box_ceiling'), 'clk', d.get('clocks'))
print('c5', d.get('config5', {}).get('ms_per_step'), 'obs', d.get('observed_checksums', {}).get('checksums_ms'))
"
PMC_RE='k_phase1|k_p2_respond|k_phase3|k_p2_apply|k_phase2' \
PMC_PASSES='SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_ACTIVE_INST_VALU' \
  bash tools/pmc.sh 65536 3 20 insts_$TAG || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_insts_$TAG 3 | tee gpurun_out/pmc_insts_$TAG.txt
