#!/bin/bash
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
AB_MODE=bench bash tools/gpu_ab.sh default pmin128 pmin2048 default pmin128 pmin2048 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03e.json 2> gpurun_out/bench_r03e.err || { tail -5 gpurun_out/bench_r03e.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_r03e.json"))
print(d["ms_per_step"], d["rounds_per_s"], d["kernel_ms"])
for k, st in d["stages"].items():
    print(k, st["avg_launch_ms"], st["frac"], st["units_per_launch"])
print("observed", d.get("observed_checksums"))
print("config1", d.get("config1"))
print("config3", d["config3"]["ms_per_step"], d["config3"]["roofline"]["frac"])
print("config5", d["config5"]["value"], d["config5"]["ms_per_step"])
print("cpu", json.dumps(d["cpu_baseline"])[:600])
PY
