#!/bin/bash
# One GPU call for an A/B step: the -m gpu suite on the in-tree library
# (any failure ends the script: only a green tree is timed), then per-kernel rocprof means of the headline bench for each
# variant (tools/gpu_ab.sh kstats, in the order given: repeat names to
# interleave), then optional WRITE_SIZE classes (WCLASS="variant ...").
# usage: tools/gpu_check_ab.sh tag variant...
set -u
TAG=$1; shift
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${NO_PYTEST:-0}" != 1 ]; then
  # (small cases first: a new kernel's fault shows on a fixture before a 65,536-node run)
  FIRST="tests/test_gpu_parity.py tests/test_gpu_node.py tests/test_gpu_wire.py tests/test_gpu_ring_incremental.py"
  FIRST="$FIRST tests/test_gpu_shards.py tests/test_gpu_rccl_selftest.py tests/test_gpu_loop_ranks.py tests/test_js.py"
  REST=$(for f in tests/test_*.py; do case " $FIRST tests/test_gpu_fullsize.py " in *" $f "*) ;; *) echo $f;; esac; done)
  FILES="$FIRST $REST tests/test_gpu_fullsize.py"
  timeout -k 10 900 python -u -m pytest $FILES -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc  # (timings only of a green tree: a failing one may fault the GPU again)
fi
[ $# -gt 0 ] && { AB_MODE=kstats bash tools/gpu_ab.sh "$@" || exit $?; }
[ -n "${WCLASS:-}" ] && { bash tools/gpu_write_classes.sh w$TAG $WCLASS || exit $?; }
exit 0
