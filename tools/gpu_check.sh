#!/bin/bash
# GPU check run used with gpurun: parity tests, then smoke; stops at the first
# crash / timeout (exit codes 124, 134, 137, 139) without starting more GPU work.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
tail -25 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?
echo "smoke exit $rc2" >> gpurun_out/smoke.log
tail -5 gpurun_out/smoke.log
exit $(( rc != 0 ? rc : rc2 ))
