set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/round_trace.py --rounds 60 --out gpurun_out/round_trace.jsonl > gpurun_out/round_trace.log 2>&1 || exit $?
RINGPOP_HIP_LIB=$PWD/ringpop_amd/libringpop_hip_diag.so timeout -k 10 200 python -u tools/diag.py > gpurun_out/diag.log 2>&1
