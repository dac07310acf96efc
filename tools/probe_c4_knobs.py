"""Config 4 (65,536 nodes, 1 % churn) ms/round for the simulation's runtime
thresholds: prefix packing (prefix_min) and log compaction (compact mul, add).
Each setting: a fresh cluster, 60 pre-roll + 5 warmup rounds, then 30 timed
rounds (as bench.py's headline, without its extras); "timing": the same with
the per-stage HIP events on (bench.py's kernel_ms).  Interleaved passes.
usage: python3 tools/probe_c4_knobs.py [passes]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ringpop_amd  # noqa: E402

SETTINGS = [
    ("default", {}),
    ("timing", {"timing": True}),
    ("prefix256", {"prefix_min": 256}),
    ("prefix1024", {"prefix_min": 1024}),
    ("prefix2048", {"prefix_min": 2048}),
    ("compact3", {"compact": (3, 8192)}),
    ("compact6", {"compact": (6, 8192)}),
]


def run(kw, n=65536, steps=30):
    kw = dict(kw)
    timing = kw.pop("timing", False)
    S = ringpop_amd.Sim(n, 2024, churn_k=656, **kw)
    S.run(65, churn=True)
    S.sync()
    S.enable_timing(timing)
    t0 = time.perf_counter()
    S.run(steps, churn=True)
    S.sync()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    S.close()
    return ms


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    sel = [(name, kw) for name, kw in SETTINGS if only is None or name in only]
    out = {name: [] for name, _ in sel}
    for _ in range(passes):
        for name, kw in sel:
            out[name].append(round(run(kw), 4))
            print(name, out[name][-1], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
