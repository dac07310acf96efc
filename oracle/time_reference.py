"""TEST INFRASTRUCTURE ONLY: time the reference JavaScript beside the oracle.

    python oracle/time_reference.py [--n 512] [--k 6] [--out bench_data/reference_js_config4.json]

Runs in the build container only (it needs /root/reference and node): the
harness (oracle/harness/sim.js) drives the reference's own modules -- index.js
RingPop, lib/*, server/* -- for N instances on one core, and the C oracle runs
the identical seeded rounds; both evaluate exactly the same changes (checked).
bench.py reports the result as `cpu_baseline.reference_js` (labelled as a
build-container measurement), and the ratio shows how far
the oracle port outruns the reference on the same inputs.
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
import oracle  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=512)
    p.add_argument("--k", type=int, default=6)
    p.add_argument("--seed", type=int, default=2024)
    p.add_argument("--rounds", type=int, default=30)
    p.add_argument("--time-from", type=int, default=10)
    p.add_argument("--out", default=os.path.join(ROOT, "bench_data", "reference_js_config4.json"))
    a = p.parse_args()
    cfg = {"n": a.n, "seed": a.seed, "churnK": a.k, "churnRounds": a.rounds, "maxRounds": a.rounds,
           "timeFrom": a.time_from, "noFinal": True}
    env = dict(os.environ, NODE_PATH=os.path.join(HERE, "harness", "shims"))
    t0 = time.time()
    r = subprocess.run(["node", "--max-old-space-size=16384", os.path.join(HERE, "harness", "sim.js"), json.dumps(cfg)],
                       env=env, capture_output=True, text=True, check=True)
    js = json.loads(r.stdout)
    wall = time.time() - t0
    t = js["timing"]
    S = oracle.Sim(a.n, a.seed, churn_k=a.k, eager=True)
    ev = 0
    for rr in range(a.rounds):
        if rr == a.time_from:
            t1 = time.perf_counter()
        o = S.round(churn=True)
        assert o["evaluated"] == js["rounds"][rr]["evaluated"], (rr, o["evaluated"], js["rounds"][rr]["evaluated"])
        if rr >= a.time_from:
            ev += o["evaluated"]
    osec = time.perf_counter() - t1
    assert ev == t["evaluated"]
    out = {
        "what": "reference ringpop JS (unmodified lib/, index.js, server/ driven by oracle/harness/sim.js) vs the C "
                "oracle on identical seeded rounds, one core each, measured in the build container",
        "node": subprocess.run(["node", "--version"], capture_output=True, text=True).stdout.strip(),
        "host": platform.processor() or platform.machine(), "cores": 1,
        "config": {"nodes": a.n, "churn_per_round": a.k, "seed": a.seed, "timed_rounds": f"{a.time_from}..{a.rounds - 1}"},
        "evaluated": t["evaluated"], "applied": t["applied"],
        "reference_js": {"seconds": round(t["seconds"], 3), "member_updates_per_s": round(t["evaluated"] / t["seconds"], 1),
                         "bootstrap_seconds": round(t["bootstrapSeconds"], 1)},
        "oracle": {"seconds": round(osec, 3), "member_updates_per_s": round(ev / osec, 1), "eager_checksums": True},
        "oracle_over_reference": round((ev / osec) / (t["evaluated"] / t["seconds"]), 2),
        "total_wall_s": round(wall, 1),
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
