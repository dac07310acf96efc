#!/bin/bash
# A/B of library variants (tools/build_variant.sh; "default" = the in-tree
# build), in the order given (repeat names to interleave runs on one box).
#   AB_MODE=kstats   (default) per-kernel rocprof means of the headline bench
#                    (tools/gpu_kstats.sh); AB_PMC=1 adds the round kernels'
#                    FETCH/WRITE bytes per launch (tools/traffic.sh)
#   AB_MODE=bench    headline bench line per variant: ms/round, kernel ms, frac
#   AB_MODE=failure  config 5 per variant: rounds, ms/round, kernel ms
#   AB_MODE=shards   config 4 on SHARDS (default 4) in-process shards: ms/round,
#                    exchange bytes per round
#   AB_MODE=diag     wg_issue section cycles (RP_DIAG variants; tools/diag.py,
#                    RP_DIAG_PHASE / RP_DIAG_FINE from the environment)
# AB_ARGS="..."      extra bench.py arguments for every run (e.g. --nodes 32768,
#                    --shards 4 with AB_MODE=failure, --loop-ranks 4)
# AB_PYTEST=1        first the -m gpu parity suite with the in-tree library
#                    (stops on a failure): a variant is only timed once the
#                    tree it came from is green
# usage: [AB_MODE=...] tools/gpu_ab.sh name ...
# (round 3's one-off experiment scripts were presets of these modes; their
# results are under profiles/r03/ab_*.txt)
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
lib_of() { if [ "$1" = default ]; then echo "$PWD/ringpop_amd/libringpop_hip.so"; else echo "$PWD/ringpop_amd/variants/libringpop_hip_$1.so"; fi; }
MODE=${AB_MODE:-kstats}
if [ "${AB_PYTEST:-0}" = 1 ]; then
  TMPDIR=/tmp timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = diag ]; then
  for v in "$@"; do
    RINGPOP_HIP_LIB=$(lib_of $v) timeout -k 10 300 python3 -u tools/diag.py ${AB_NODES:-65536} > gpurun_out/diag_$v.json 2>&1 \
      || { echo "$v failed"; tail -3 gpurun_out/diag_$v.json; exit 1; }
    echo "== $v"; cat gpurun_out/diag_$v.json
  done
  exit 0
fi
if [ "$MODE" = kstats ]; then
  bash tools/gpu_kstats.sh "$@" || exit $?
  [ "${AB_PMC:-0}" = 1 ] || exit 0
  for v in "$@"; do
    RINGPOP_HIP_LIB=$(lib_of $v) bash tools/traffic.sh 65536 10 5 ab_$v > /dev/null || { echo "$v pmc failed"; exit 1; }
    echo "== $v traffic"
    python3 -c "
import json; d = json.load(open('gpurun_out/traffic_ab_$v/traffic_ab_$v.json'))
for k, x in d.items():
    if 'fetch_kib_raw' in x: print(f\"{k:14s} x{x['launches_per_round']} fetch*2 {2*x['fetch_kib_raw']*1024/1e9:.3f} GB  write {x['write_kib']*1024/1e9:.3f} GB per launch\")
"
  done
  exit 0
fi
for v in "$@"; do
  case $MODE in
    bench) ARGS="--no-cpu-baseline --no-extras --no-traffic" ;;
    failure) ARGS="--workload failure --no-cpu-baseline" ;;
    shards) ARGS="--shards ${SHARDS:-4} --no-extras --no-cpu-baseline --no-traffic" ;;
    *) echo "unknown AB_MODE $MODE"; exit 2 ;;
  esac
  RINGPOP_HIP_LIB=$(lib_of $v) timeout -k 10 300 python -u bench.py $ARGS ${AB_ARGS:-} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  rc=$?
  python3 -c "
import json; d = json.load(open('gpurun_out/ab_$v.json'))
print('$v', d['value'], d['ms_per_step'], d['kernel_ms'], (d.get('roofline') or {}).get('frac'), d.get('exchange'))
" || { echo "$v failed rc=$rc"; tail -3 gpurun_out/ab_$v.err; exit 1; }
done
