#!/bin/bash
# the rank path timed on one GPU (loopback transport): config 4 and config 5 on 4 ranks, beside the in-process shards
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --loop-ranks 4 --no-cpu-baseline > gpurun_out/za_c4_loop4.json 2> gpurun_out/za_c4_loop4.err || { echo c4 loop failed; tail -5 gpurun_out/za_c4_loop4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/za_c4_loop4.json')); print('c4 loop4', d['ms_per_step'], d['exchange']['bytes_per_round_max_rank'])"
timeout -k 10 300 python -u bench.py --shards 4 --no-cpu-baseline --no-extras > gpurun_out/za_c4_sh4.json 2> gpurun_out/za_c4_sh4.err || { echo c4 sh4 failed; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/za_c4_sh4.json')); print('c4 sh4', d['ms_per_step'], d['exchange']['bytes_per_round_max_rank'])"
timeout -k 10 300 python -u bench.py --workload failure --nodes 32768 --loop-ranks 4 --no-cpu-baseline > gpurun_out/za_f32_loop4.json 2> gpurun_out/za_f32_loop4.err || { echo f32 loop failed; tail -5 gpurun_out/za_f32_loop4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/za_f32_loop4.json')); print('c5 32k loop4', d['value'], d['ms_per_step'], d['exchange']['bytes_per_round_max_rank'])"
timeout -k 10 400 python -u bench.py --workload failure --loop-ranks 4 --no-cpu-baseline > gpurun_out/za_f64_loop4.json 2> gpurun_out/za_f64_loop4.err || { echo f64 loop failed; tail -5 gpurun_out/za_f64_loop4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/za_f64_loop4.json')); print('c5 64k loop4', d['value'], d['ms_per_step'], d['exchange']['bytes_per_round_max_rank'])"
