"""Per-round trajectory of the device simulation: wall time per round and the
work counters, to see where the steady state begins.

usage: python tools/round_trace.py [--nodes N] [--rounds R] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from ringpop_amd.sim import Sim  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=120)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--out", default="gpurun_out/round_trace.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    t0 = time.time()
    sim = Sim(a.nodes, a.seed)
    sim.sync()
    print(f"setup {time.time() - t0:.2f}s", flush=True)
    prev = sim.counters()
    with open(a.out, "w") as f:
        for r in range(a.rounds):
            t = time.perf_counter()
            sim.run(1)
            sim.sync()
            ms = (time.perf_counter() - t) * 1e3
            cur = sim.counters()
            d = {k: cur[k] - prev[k] for k in cur}
            prev = cur
            d["round"] = r
            d["ms"] = round(ms, 3)
            f.write(json.dumps(d) + "\n")
            f.flush()
            if r % 10 == 0 or r == a.rounds - 1:
                print(f"r{r:4d} {ms:8.2f} ms eval={d['evaluated']:.3e} applied={d['applied']:.3e} "
                      f"scan1={d['scanned_send_issue']:.3e} emit1={d['emitted_send_issue']:.3e} "
                      f"conv={d['converged_rounds']}", flush=True)
    sim.close()


if __name__ == "__main__":
    main()
