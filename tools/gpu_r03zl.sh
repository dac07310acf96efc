#!/bin/bash
# first-run penalty: bench with a device prewarm as the box's first process, then without, then with
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for v in 3 0 3 0; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-extras --prewarm $v > gpurun_out/pw_$v.json 2> gpurun_out/pw_$v.err || { echo "prewarm $v failed"; tail -3 gpurun_out/pw_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/pw_$v.json'));print('prewarm $v', d['ms_per_step'], {k:v['avg_launch_ms'] for k,v in d['stages'].items()})"
done
