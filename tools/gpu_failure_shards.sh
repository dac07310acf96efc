set -e
cd $GRAFT_REPO_ROOT
for s in 1 4; do
  timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --shards $s --no-cpu-baseline > gpurun_out/f32_sh$s.json 2> gpurun_out/f32_sh$s.err
  python3 -c "import json; d=json.load(open('gpurun_out/f32_sh$s.json')); print($s, d['value'], d['ms_per_step'], d['kernel_ms'], d.get('exchange'))"
done
timeout -k 10 300 python -u bench.py --workload failure --shards 4 --no-cpu-baseline > gpurun_out/f64_sh4.json 2> gpurun_out/f64_sh4.err
python3 -c "import json; d=json.load(open('gpurun_out/f64_sh4.json')); print('64k/4', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('exchange'))"
timeout -k 10 300 python -u bench.py --workload failure --no-cpu-baseline > gpurun_out/f64_sh1.json 2> gpurun_out/f64_sh1.err
python3 -c "import json; d=json.load(open('gpurun_out/f64_sh1.json')); print('64k/1', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('exchange'))"
