#!/usr/bin/env python3
"""Headline benchmark: gossip rounds of a 65,536-node simulated ringpop cluster.

    python bench.py [--gpus N] [--steps K] [--warmup W]

A step is one gossip round (every live node pings once: iterator, piggyback
issue, receiver merge + response, sender merge) of config 4:
65,536 nodes with full views, ceil(1% N) = 656 alive re-assertions per round.
value = member-updates/s (changes evaluated by Membership.update, all ranks),
with rounds/s alongside.  Inputs are resident in HBM before timing.

N > 1 (torchrun, one rank per GPU): each rank runs its own 65,536-node
cluster (replicas; the sharded RCCL exchange is future work),
so per-GPU work is fixed and scaling is "weak".
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "gossip rounds/sec (member-updates/s) at 65,536 sim nodes, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# SURVEY.md §8(d) algorithmic bytes: merge = 16 B change + 16 B view entry per
# evaluated change, + 16 B entry write + 16 B dissemination record per applied.
MERGE_B_EVAL, MERGE_B_APPLIED = 32, 32


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--nodes", type=int, default=65536)
    p.add_argument("--churn", type=int, default=None, help="alive re-assertions per round (default ceil(1%% N))")
    p.add_argument("--seed", type=int, default=2024)
    p.add_argument("--cpu-nodes", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"))
    return p.parse_args()


def cpu_baseline(args):
    """Oracle (C restatement, reference-faithful eager checksums), one host core,
    on a bounded sample of the same workload shape."""
    import oracle
    oracle.build()
    n = args.cpu_nodes
    k = math.ceil(0.01 * n)
    S = oracle.Sim(n, args.seed, churn_k=k, eager=True)
    for _ in range(8):
        S.round(churn=True)
    ev, t0, rounds = 0, time.perf_counter(), 0
    while True:
        ev += S.round(churn=True)["evaluated"]
        rounds += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or rounds >= 200:
            break
    S.close()
    return {"value": ev / el, "unit": "member-updates/s", "cores": 1, "kind": "port",
            "sample": f"oracle/sim_oracle.c, {n} nodes, {k} re-assertions/round, {rounds} steady-state rounds "
                      f"after 8 warmup rounds ({el:.1f} s, eager checksums as the reference computes them)",
            "rounds_per_s": rounds / el}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    import ringpop_amd
    from ringpop_amd import build
    from ringpop_amd._lib import check, lib
    if rank == 0 or world == 1:
        build.build()
    if dist:
        dist.barrier()
    check(lib().rp_set_device(local))

    n = args.nodes
    k = args.churn if args.churn is not None else math.ceil(0.01 * n)
    S = ringpop_amd.Sim(n, args.seed + rank, churn_k=k)
    S.run(args.warmup, churn=True)
    S.sync()
    c0 = S.counters()

    def barrier():
        if dist:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    S.enable_timing(True)
    barrier()
    t0 = time.perf_counter()
    S.run(args.steps, churn=True)
    S.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    c1 = S.counters()
    kt = S.kernel_times()
    d = {key: c1[key] - c0[key] for key in c1}

    if dist:
        import torch
        t = torch.tensor([elapsed, float(d["evaluated"]), float(d["applied"])], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0].item())
        total_eval = float(t[1].item())
        total_applied = float(t[2].item())
    else:
        total_eval, total_applied = float(d["evaluated"]), float(d["applied"])

    if rank != 0:
        S.close()
        if dist:
            dist.destroy_process_group()
        return

    # dominant kernel: the sender-side response merge (k_phase3) or the ping
    # merge (k_phase2), whichever spent more device time
    cand = {
        "merge_resp": (kt["merge_resp"], d["eval_resp_merge"], d["applied_resp_merge"], "k_phase3"),
        "merge_ping": (kt["merge_ping"], d["eval_ping_merge"], d["applied_ping_merge"], "k_phase2"),
    }
    name = max(cand, key=lambda c: cand[c][0][0])
    (ms, launches), ev, ap, kname = cand[name]
    alg_bytes = MERGE_B_EVAL * ev + MERGE_B_APPLIED * ap
    per_launch_s = (ms / 1000.0) / max(launches, 1)
    achieved = alg_bytes / max(launches, 1) / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get(kname, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kname,
                "algorithmic_bytes_per_launch": int(alg_bytes / max(launches, 1)),
                "avg_launch_ms": round(per_launch_s * 1e3, 4)}

    value = total_eval / elapsed
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "member-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"config 4: {n} simulated ringpop nodes, full views, {k} alive re-assertions/round, "
                               "steady-state gossip rounds",
                   "nodes": n, "churn_per_round": k, "seed": args.seed,
                   "parallelism": "replicas" if world > 1 else "single"},
        "rounds_per_s": round(args.steps * world / elapsed, 3),
        "applied_per_s": round(total_applied / elapsed, 1),
        "kernel_ms": {c: round(v[0], 3) for c, v in kt.items()},
        "roofline": roofline,
    }
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(args)
    S.close()
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
