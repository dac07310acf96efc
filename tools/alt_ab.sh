set -u
for i in 1 2; do for v in default old; do
  if [ $v = default ]; then L=$PWD/ringpop_amd/libringpop_hip.so; else L=$PWD/ringpop_amd/variants/libringpop_hip_$v.so; fi
  RINGPOP_HIP_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/alt.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/alt.json')); print('$v', d['ms_per_step'], d['kernel_ms']['merge_ping'], d['roofline']['frac'])"
done; done
