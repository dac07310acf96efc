#!/usr/bin/env python3
"""Headline benchmark: gossip rounds of a 65,536-node simulated ringpop cluster.

    python bench.py [--gpus N] [--steps K] [--warmup W]

A step is one gossip round (every live node pings once: iterator, piggyback
issue, receiver merge + response, sender merge) of config 4:
65,536 nodes with full views, ceil(1% N) = 656 alive re-assertions per round.
The cluster is first pre-rolled --preroll rounds (default 60) so that every
node's dissemination log holds its steady-state load whatever --warmup is.
value = member-updates/s (changes passed to Membership.update, the
reference's accounting, all ranks); beside it rounds/s, the changes whose
view cell was physically read (`touched`, after the sender and seen filters)
and applied/s.  Inputs are resident in HBM before timing.

N = 1 also runs, after the headline, config 3 (100 M string keys vs a
10,000-server ring: keys/s, roofline, sampled parity) and config 5 (10 %
fail-stops + a false-suspicion storm at 65,536 nodes: rounds to converge,
ms/round, end-state checks), reported as sub-objects of the same JSON line,
and the CPU baselines.

N > 1 (torchrun, one rank per GPU): the 65,536 nodes are sharded over the
ranks (N/G consecutive ids each); every round the shards exchange ping
metadata, checksum snapshots, ping bodies and responses with RCCL all-gathers
and send/recv groups inside libringpop_hip.  Total work is
fixed, so scaling is "strong"; value is the cluster's member-updates/s.
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
# `evaluated` counts the reference's list lengths; the seen filter leaves ~95 %
# of them out of the messages (provable no-ops), so these "reference
# equivalent" bytes are not work done: the roofline's numerator
# is the work bytes below, the reference-equivalent figure a separate field.
MERGE_B_EVAL, MERGE_B_APPLIED = 32, 32
# Work bytes of a merge / issue stage: 16 B change + 16 B view cell per change
# read against a view cell (touched), 16 B cell + 16 B log record written per
# applied change, 4 B per dissemination-log word an issue scans, 16 B per
# change it writes out.
WORK_B_TOUCHED, WORK_B_APPLIED, WORK_B_SCANNED, WORK_B_WRITTEN = 32, 32, 4, 16
REFERENCE_JS = os.path.join(ROOT, "bench_data", "reference_js_config4.json")
# The ceiling of the merges' dominant access, measured (tools/micro/fetch_cal.hip,
# profiles/r04/fetch_cal_r04n.json): random 16-byte read + 8-byte write-back
# of cells in 1 MB rows spread over 32 GB, 24.9 G accesses/s on one MI355X
# (each one a 128-byte line fetched and a 32-byte sector written).
RANDOM_RMW_PEAK = 24.9e9


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--preroll", type=int, default=60, help="rounds run before warmup to reach the steady log fill")
    p.add_argument("--nodes", type=int, default=65536)
    p.add_argument("--churn", type=int, default=None, help="alive re-assertions per round (default ceil(1%% N))")
    p.add_argument("--seed", type=int, default=2024)
    p.add_argument("--cpu-nodes", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-all-cores", action="store_true", help="cpu_baseline: skip the 16-replica oracle sample")
    p.add_argument("--no-extras", action="store_true", help="N=1: skip the config-3 and config-5 sub-benchmarks")
    p.add_argument("--no-traffic", action="store_true",
                   help="N=1: skip the rocprofv3 FETCH_SIZE / WRITE_SIZE child runs behind roofline.traffic")
    p.add_argument("--shards", type=int, default=1, help="N=1: split the cluster into this many in-process shards")
    p.add_argument("--loop-ranks", type=int, default=0,
                   help="N=1: run the cluster as this many ranks of the RCCL rank code, host threads of this "
                        "process exchanging through the loopback transport (rp_sim_create_rank_loop)")
    p.add_argument("--workload", choices=("gossip", "lookup", "failure"), default="gossip",
                   help="gossip: config 4 (headline); lookup: config 3; failure: config 5 rounds-to-converge")
    p.add_argument("--keys", type=int, default=100_000_000, help="lookup: keys per batch")
    p.add_argument("--servers", type=int, default=10_000, help="lookup: ring servers (x100 replica points)")
    p.add_argument("--fail-frac", type=float, default=0.10, help="failure: fraction of nodes fail-stopped at round 0")
    p.add_argument("--storm-ppm", type=int, default=1000, help="failure: false suspicions per round, ppm of live nodes")
    p.add_argument("--storm-rounds", type=int, default=20, help="failure: rounds of the false-suspicion storm")
    p.add_argument("--max-rounds", type=int, default=400, help="failure: give up after this many rounds")
    return p.parse_args(argv)


# ----------------------------------------------------------------- CPU baselines
def _oracle_rate(n, seed, seconds, eager=True):
    """The oracle (C restatement) on one core: steady-state member-updates/s
    of an n-node cluster.  eager: a farmhash checksum after every applied
    batch, as the reference computes it (lib/membership.js:266-268); lazy:
    only the checksums the protocol reads (the device's policy)."""
    import oracle
    k = math.ceil(0.01 * n)
    S = oracle.Sim(n, seed, churn_k=k, eager=eager)
    for _ in range(8):
        S.round(churn=True)
    ev, rounds, t0 = 0, 0, time.perf_counter()
    while True:
        ev += S.round(churn=True)["evaluated"]
        rounds += 1
        el = time.perf_counter() - t0
        if el >= seconds or rounds >= 200:
            break
    S.close()
    return ev / el, rounds, el, k


def _oracle_rate_replicas(n, seed, seconds, procs):
    """The same oracle sample in `procs` independent processes at once (one
    cluster each; the restatement is sequential by definition, like the
    reference's event loop): aggregate member-updates/s of the host's cores.
    Children are fresh interpreters that never touch the GPU."""
    import subprocess
    code = ("import json, sys; sys.path.insert(0, %r); import bench; "
            "r, rounds, el, k = bench._oracle_rate(%d, %d, %f); print(json.dumps([r, rounds, el]))"
            % (os.path.dirname(os.path.abspath(__file__)), n, seed, seconds))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           env=env) for _ in range(procs)]
    rates = []
    for p in ps:
        out, err = p.communicate(timeout=seconds * 4 + 120)
        if p.returncode != 0:
            raise RuntimeError("oracle replica failed: " + err[-500:])
        rates.append(json.loads(out.strip().splitlines()[-1])[0])
    return sum(rates), rates


def cpu_baseline(args, gpu_eval_per_round):
    """SURVEY.md §8(d) CPU timing beside the GPU:
    (1) the oracle port on one core of this host at two sizes, extrapolated to
        65,536 nodes through its measured cost per evaluated change;
    (2) the reference JavaScript itself, measured in the build container on the
        same seeded inputs as the oracle (bench_data/reference_js_config4.json; the
        reference cannot travel to the GPU box)."""
    import oracle
    oracle.build()
    n1, n2 = args.cpu_nodes // 2, args.cpu_nodes
    r1, _, _, _ = _oracle_rate(n1, args.seed, args.cpu_seconds / 2)
    r2, rounds, el, k = _oracle_rate(n2, args.seed, args.cpu_seconds)
    # cost per evaluated change c(N) = 1/rate, linear in N (each applied batch
    # re-renders an N-member checksum string): c(N) = a + b N through both samples
    c1, c2 = 1.0 / r1, 1.0 / r2
    b = (c2 - c1) / (n2 - n1)
    a = c1 - b * n1
    c65 = a + b * args.nodes
    rl, rounds_l, el_l, _ = _oracle_rate(n2, args.seed, args.cpu_seconds / 2, eager=False)
    out = {"value": round(r2, 1), "unit": "member-updates/s", "cores": 1, "kind": "port",
           "sample": f"oracle/sim_oracle.c on 1 host core, {n2} nodes, {k} re-assertions/round, {rounds} steady-state "
                     f"rounds after 8 warmup rounds ({el:.1f} s, eager checksums as the reference computes them)",
           "at_nodes": {str(n1): round(r1, 1), str(n2): round(r2, 1)},
           "lazy_checksums": {"value": round(rl, 1), "unit": "member-updates/s", "cores": 1, "nodes": n2,
                              "sample": f"the same oracle computing only the checksums the protocol reads (the "
                                        f"device's policy): {rounds_l} rounds in {el_l:.1f} s"},
           "extrapolated_65536": {
               "member_updates_per_s": round(1.0 / c65, 1),
               "rounds_per_s": round(1.0 / (c65 * gpu_eval_per_round), 5) if gpu_eval_per_round else None,
               "formula": f"cost per evaluated change c(N) = a + b*N fitted at N={n1},{n2} "
                          f"(a={a:.3e} s, b={b:.3e} s/node); rounds/s = 1 / (c(65536) x the GPU run's evaluated "
                          f"changes per round, {gpu_eval_per_round:.4g})"}}
    procs = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16 cores
    if procs > 1 and not args.no_all_cores:
        agg, rates = _oracle_rate_replicas(n2, args.seed, args.cpu_seconds / 2, procs)
        out["replicas_16"] = {"value": round(agg, 1), "unit": "member-updates/s", "cores": procs, "kind": "port",
                              "nproc": os.cpu_count(),
                              "sample": f"{procs} independent replicas: {procs} oracle processes at once, each its "
                                        f"own {n2}-node cluster (the sample above) for {args.cpu_seconds / 2:.0f} s; "
                                        f"summed rate of {procs} clusters, not one cluster on {procs} cores (the "
                                        f"restatement, like the reference's event loop, is sequential per cluster); "
                                        f"{procs} = this job's CPU share of the GPU box, of nproc = {os.cpu_count()}",
                              "per_process": [round(x, 1) for x in rates]}
    if os.path.exists(REFERENCE_JS):
        js = json.load(open(REFERENCE_JS))
        out["reference_js"] = {
            "value": js["reference_js"]["member_updates_per_s"], "unit": "member-updates/s", "cores": 1,
            "kind": "reference", "measured": "in the build container (node " + js["node"] + "), not on the GPU box: "
            "the reference's unmodified lib/ and server/ driven by oracle/harness/sim.js",
            "nodes": js["config"]["nodes"], "oracle_over_reference": js["oracle_over_reference"],
            "extrapolated_65536_member_updates_per_s": round(1.0 / c65 / js["oracle_over_reference"], 1),
            "formula": "oracle extrapolation / (oracle-over-reference ratio measured on identical inputs at "
                       f"{js['config']['nodes']} nodes)"}
    return out


# ----------------------------------------------------------------- this box's ceilings
CAL_BYTES = 16 << 30  # rp_calibrate's allocation: 64x the Infinity Cache


def box_ceiling():
    """This box's own ceilings for the round kernels' access kinds, measured
    in-process right before the cluster is built (rp_calibrate: random 16-B
    reads, random 16-B read + 8-B write-backs, random 4-B reads, 16-B and 4-B
    per lane streaming over 16 GiB): the same build runs several percent
    apart on different boxes, so each stage is also reported as a
    fraction of the box it ran on."""
    import ctypes

    from ringpop_amd._lib import check, lib
    v = (ctypes.c_double * 5)()
    t0 = time.perf_counter()
    check(lib().rp_calibrate(CAL_BYTES, v, 5))
    ms = (time.perf_counter() - t0) * 1e3
    return {"rand16_per_s": round(v[0], 1), "rand16_rmw_per_s": round(v[1], 1), "rand4_per_s": round(v[2], 1),
            "stream16_GBps": round(v[3] * 16 / 1e9, 2), "stream4_words_per_s": round(v[4], 1),
            "stream4_GBps": round(v[4] * 4 / 1e9, 2), "bytes": CAL_BYTES, "wall_ms": round(ms, 1),
            "method": "rp_calibrate (ringpop_amd/csrc/rp_calib.hip): 537 M accesses per launch, 2 timed launches "
                      "per kind after an untimed one, HIP events, before the cluster is built"}


def _pci_bus_id():
    import ctypes

    from ringpop_amd._lib import lib
    b = ctypes.create_string_buffer(64)
    if lib().rp_device_pci_bus_id(b, 64) != 0:
        return None
    return b.value.decode().lower()


def _dpm_now(path):
    """The current level of a pp_dpm_* file (the line marked '*'), in MHz."""
    try:
        with open(path) as f:
            for line in f:
                if "*" in line:
                    tok = line.split(":", 1)[1].replace("*", "").strip().lower()
                    return float(tok.replace("mhz", "").strip())
    except (OSError, ValueError, IndexError):
        return None
    return None


class ClockSampler:
    """sclk / mclk / fclk of this process's GPU from sysfs (pp_dpm_*, read
    without HIP) sampled on a host thread while the timed region runs, and
    once before and after it."""

    def __init__(self, bus_id):
        self.dev = f"/sys/bus/pci/devices/{bus_id}" if bus_id else None
        self.samples = []
        self._stop = None
        self._th = None

    def read(self):
        if not self.dev:
            return {}
        return {k: _dpm_now(os.path.join(self.dev, "pp_dpm_" + k)) for k in ("sclk", "mclk", "fclk")}

    def start(self):
        import threading
        self.before = self.read()
        self._stop = threading.Event()

        def loop():
            while not self._stop.is_set():
                self.samples.append(self.read())
                self._stop.wait(0.01)
        self._th = threading.Thread(target=loop, daemon=True)
        self._th.start()

    def stop(self):
        if self._th:
            self._stop.set()
            self._th.join(timeout=5)
        self.after = self.read()

    def report(self):
        out = {"sysfs": self.dev, "before": getattr(self, "before", {}), "after": getattr(self, "after", {})}
        for k in ("sclk", "mclk", "fclk"):
            xs = [s[k] for s in self.samples if s.get(k) is not None]
            if xs:
                out[k + "_during_MHz"] = {"min": min(xs), "max": max(xs), "mean": round(sum(xs) / len(xs), 1),
                                          "samples": len(xs)}
        return out


def frac_of_box(stage, box):
    """A stage against this box's measured ceilings: its work bytes against
    16-B streaming, its applied / touched changes against the random cell
    read-modify-write / read rates, its scanned log words against 4-B
    streaming."""
    per_s = stage["avg_launch_ms"] / 1e3
    if not per_s or not box:
        return None
    u = stage["units_per_launch"]
    out = {"work_over_stream16": round(stage["work_bytes_per_launch"] / per_s / 1e9 / box["stream16_GBps"], 4)}
    if u.get("applied"):
        out["applied_over_rand16_rmw"] = round(u["applied"] / per_s / box["rand16_rmw_per_s"], 4)
    if u.get("touched"):
        out["touched_over_rand16"] = round(u["touched"] / per_s / box["rand16_per_s"], 4)
    if u.get("log_words_scanned"):
        out["scanned_over_stream4"] = round(u["log_words_scanned"] / per_s / box["stream4_words_per_s"], 4)
    return out


# ----------------------------------------------------------------- HBM traffic (PMC)
TRAFFIC_KERNELS = {"ping_merge": ("k_p2_lists", "k_p2_apply", "k_p2_respond", "k_phase2"),
                   "resp_merge": ("k_phase3",), "send_issue": ("k_iterate", "k_shuffle", "k_phase1")}


def _pmc_rows(counters, regex, child_args, outdir):
    """One rocprofv3 --pmc pass (no tracing) over a child run of this script:
    {kernel: [(dispatch id, {counter: value})]}."""
    import csv
    import shutil
    import subprocess
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    cmd = [rp, "--pmc", *counters, "--kernel-include-regex", regex, "-d", outdir, "-o", "run", "--output-format",
           "csv", "--", sys.executable, os.path.abspath(__file__), *child_args]
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 --pmc {counters} exit {r.returncode}: {r.stderr[-300:]}")
    path = None
    for root, _, files in os.walk(outdir):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(root, f)
    if not path:
        raise RuntimeError(f"rocprofv3 --pmc {counters}: no counter_collection.csv")
    per = {}
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
        per.setdefault(name, {}).setdefault(int(row["Dispatch_Id"]), {})[row["Counter_Name"]] = float(row["Counter_Value"])
    return {k: sorted(v.items()) for k, v in per.items()}


def lookup_pmc(args):
    """Config 3's k_lookup_keys under two --pmc passes (FETCH_SIZE; the L2's
    hits and misses): bytes and L2 misses per key, for its bound label."""
    import tempfile
    d = tempfile.mkdtemp(prefix="rp_pmc_lk_")
    child = ["--workload", "lookup", "--steps", "2", "--warmup", "1", "--keys", str(args.keys), "--servers",
             str(args.servers), "--no-cpu-baseline"]
    f = _pmc_rows(["FETCH_SIZE"], "k_lookup_keys", child, os.path.join(d, "f"))
    h = _pmc_rows(["TCC_HIT_sum", "TCC_MISS_sum"], "k_lookup_keys", child, os.path.join(d, "h"))
    fr = [c["FETCH_SIZE"] for _, c in next(v for k, v in f.items() if "k_lookup_keys" in k)]
    hr = [c for _, c in next(v for k, v in h.items() if "k_lookup_keys" in k)]
    fetch = 2 * 1024 * sum(fr) / len(fr)
    hits = sum(c.get("TCC_HIT_sum", 0.0) for c in hr) / len(hr)
    miss = sum(c.get("TCC_MISS_sum", 0.0) for c in hr) / len(hr)
    return {"traffic": int(fetch), "l2_hits_per_key": round(hits / args.keys, 3),
            "l2_misses_per_key": round(miss / args.keys, 3),
            "method": "rocprofv3 --pmc FETCH_SIZE, then --pmc TCC_HIT_sum TCC_MISS_sum, child runs of "
                      "bench.py --workload lookup; 2 x FETCH_SIZE per launch"}


def _pmc_child(args, counter, outdir):
    """One rocprofv3 --pmc pass (a single counter, no tracing) over a short
    config-4 run of this script: the round kernels' counter per dispatch."""
    import csv
    import shutil
    import subprocess
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    regex = "|".join(k for ks in TRAFFIC_KERNELS.values() for k in ks)
    rounds = args.preroll + 6  # (the timed 3 rounds and the 3-round per-stage pass after them)
    cmd = [rp, "--pmc", counter, "--kernel-include-regex", regex, "-d", outdir, "-o", "run", "--output-format", "csv",
           "--", sys.executable, os.path.abspath(__file__), "--nodes", str(args.nodes), "--steps", "3", "--warmup", "0",
           "--preroll", str(args.preroll), "--no-extras", "--no-cpu-baseline", "--no-traffic"]
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 --pmc {counter} exit {r.returncode}: {r.stderr[-300:]}")
    path = None
    for root, _, files in os.walk(outdir):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(root, f)
    if not path:
        raise RuntimeError(f"rocprofv3 --pmc {counter}: no counter_collection.csv")
    per = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
        per.setdefault(name, []).append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    out = {}
    for name, rows in per.items():
        rows.sort()
        lpr = max(1, round(len(rows) / rounds))  # launches per round
        last = rows[-3 * lpr:]
        out[name] = {"kib_per_round": sum(v for _, v in last) / 3.0, "launches_per_round": lpr}
    return out


def attach_traffic(out, traffic):
    """roofline.traffic (and stages.*.traffic): HBM bytes per launch from
    the PMC passes; beside each, the physical rate as a fraction of peak."""
    out["traffic_pmc"] = {k: v for k, v in traffic.items() if k != "stages"} if "stages" in traffic else traffic
    if "stages" not in traffic:
        return
    for name, st in out.get("stages", {}).items():
        t = traffic["stages"].get(name)
        if not t:
            continue
        b = t["bytes_per_round"]  # (one launch of a stage per round)
        st["traffic"] = b
        st["traffic_frac"] = round(b / (st["avg_launch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if st["avg_launch_ms"] else None
        st["traffic_over_work"] = round(b / st["work_bytes_per_launch"], 3) if st["work_bytes_per_launch"] else None
        box = out.get("box_ceiling")
        if box and st["avg_launch_ms"] and st.get("frac_of_box") is not None:
            st["frac_of_box"]["traffic_over_stream16"] = round(
                b / (st["avg_launch_ms"] / 1e3) / 1e9 / box["stream16_GBps"], 4)
    r = out.get("roofline")
    if r and r.get("stage") in out.get("stages", {}):
        s = out["stages"][r["stage"]]
        r["traffic"] = b = s.get("traffic")
        r["traffic_frac"] = (round(b / (r["avg_launch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                             if b and r.get("avg_launch_ms") else s.get("traffic_frac"))
        r["traffic_over_work"] = (round(b / r["work_bytes_per_launch"], 3)
                                  if b and r.get("work_bytes_per_launch") else s.get("traffic_over_work"))
        box = out.get("box_ceiling")
        if box and b and r.get("avg_launch_ms") and r.get("frac_of_box") is not None:
            r["frac_of_box"]["traffic_over_stream16"] = round(b / (r["avg_launch_ms"] / 1e3) / 1e9 / box["stream16_GBps"], 4)


def pmc_traffic(args):
    """HBM bytes per round of each stage of the line, from two rocprofv3
    --pmc passes (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md's
    rocprofv3 section) over child runs of this same script and library,
    before this process touches the GPU; the steady state's last 3 of
    preroll + 6 rounds.  Bytes = 2 x FETCH_SIZE (the guide's gfx950
    correction, checked for this path's random 16-byte cells and 4-byte words
    by tools/micro/fetch_cal.hip) + WRITE_SIZE, KiB -> bytes."""
    import tempfile
    d = tempfile.mkdtemp(prefix="rp_pmc_")
    f = _pmc_child(args, "FETCH_SIZE", os.path.join(d, "fetch"))
    w = _pmc_child(args, "WRITE_SIZE", os.path.join(d, "write"))
    stages = {}
    for st, ks in TRAFFIC_KERNELS.items():
        fb = sum(v["kib_per_round"] for k, v in f.items() if any(x in k for x in ks))
        wb = sum(v["kib_per_round"] for k, v in w.items() if any(x in k for x in ks))
        stages[st] = {"fetch_kib_raw": round(fb, 1), "write_kib": round(wb, 1),
                      "bytes_per_round": int((2 * fb + wb) * 1024)}
    return {"stages": stages, "kernels_fetch": f, "kernels_write": w,
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate child runs of this bench, "
                      f"--preroll {args.preroll} --steps 3), last 3 rounds; 2 x FETCH_SIZE + WRITE_SIZE"}


# ----------------------------------------------------------------- config 3
def ring_names(count):
    """Server addresses of the sim's scheme (10.<b2>.<b1>.<b0>:<3000+i%7>)."""
    return [f"10.{(i >> 16) & 255}.{(i >> 8) & 255}.{i & 255}:{3000 + i % 7}" for i in range(count)]


def run_lookup(args, with_cpu=True):
    """Config 3: batched ring.lookup of device-resident keys against a
    servers x 100 replica-point ring (lib/ring.js:138-147).  A step is one
    lookup of the whole key batch; value = keys/s.  Keys, offsets and the
    owner output are resident in HBM; HIP events on the launch stream."""
    import ctypes

    import numpy as np

    import ringpop_amd
    from ringpop_amd import hiprt
    from ringpop_amd._lib import check, lib
    L = lib()
    names = ring_names(args.servers)
    # ring build (addRemoveServers of every server: 100 replica hashes each,
    # the stable radix sort of the points, first-inserter dedupe, the lookup
    # directories): host wall clock and the device time of the same call
    # (rp_ring_build_ms: HIP events around its device work)
    build_ms, build_dev_ms = [], []
    for _ in range(3):
        r0 = ringpop_amd.HashRing()
        t0 = time.perf_counter()
        assert r0.addRemoveServers(names, None)
        build_ms.append((time.perf_counter() - t0) * 1e3)
        dms = ctypes.c_double(0.0)
        check(L.rp_ring_build_ms(r0._h, ctypes.byref(dms)))
        build_dev_ms.append(dms.value)
        r0.close()
    ring = ringpop_amd.HashRing()
    assert ring.addRemoveServers(names, None)
    pts_h, pts_o = ring.points()
    d_bytes, d_off, total = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    check(L.rp_ring_make_keys_device(ring._h, args.seed, args.keys, ctypes.byref(d_bytes), ctypes.byref(d_off),
                                     ctypes.byref(total)))
    owners = hiprt.DeviceArray(args.keys, np.int32)
    stream = hiprt.Stream()

    def launch():
        check(L.rp_ring_lookup_batch_device(ring._h, d_bytes, d_off, args.keys, owners.ptr, stream.handle))

    for _ in range(max(args.warmup, 1)):
        launch()
    stream.synchronize()
    ev = [(hiprt.Event(), hiprt.Event()) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        launch()
        b.record(stream)
    stream.synchronize()
    elapsed = time.perf_counter() - t0
    kms = sum(a.elapsed_ms(b) for a, b in ev) / len(ev)
    for a, b in ev:
        a.destroy()
        b.destroy()

    # parity on a sample: oracle farmhash32 + numpy lower bound over the
    # oracle's own replica points (checker only, outside the timed region)
    import oracle
    oh, oo = oracle.ring_points_add_only(names)
    assert np.array_equal(oh, pts_h) and np.array_equal(oo, pts_o), "ring points differ from the oracle"
    rng = np.random.default_rng(args.seed)
    idx = np.unique(rng.integers(0, args.keys, size=200_000))
    keys = oracle.lookup_keys(args.seed, idx)
    want = oracle.ring_lookup_points(oh, oo, oracle.farmhash32_batch(keys))
    own_all = owners.numpy()
    got = own_all[idx]
    mismatches = int((got != want).sum())
    assert mismatches == 0, f"{mismatches} lookup owners differ from the oracle"

    # handleOrProxyAll's grouping (index.js:636-645) of the same batch on the
    # device: owner-sorted runs, first-appearance group order
    n = args.keys
    dests = hiprt.DeviceArray(n, np.int32)
    goff = hiprt.DeviceArray(n + 1, np.int32)
    kidx = hiprt.DeviceArray(n, np.int32)
    ng = ctypes.c_size_t(0)

    def group():
        check(L.rp_ring_group_device(ring._h, owners.ptr, n, dests.ptr, goff.ptr, kidx.ptr, ctypes.byref(ng),
                                     stream.handle))
    group()
    stream.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        group()
    group_ms = (time.perf_counter() - t0) * 1e3 / 3
    # the groupBy result is unique given the owners: a partition of the key
    # indices by owner, ascending within a group, groups by first key index
    g = ng.value
    d, off, ki = dests.numpy()[:g], goff.numpy()[: g + 1].astype(np.int64), kidx.numpy()
    lens = np.diff(off)
    ok = (off[0] == 0 and off[-1] == n and (lens > 0).all() and len(np.unique(d)) == g
          and np.array_equal(own_all[ki], np.repeat(d, lens))
          and (np.diff(ki[off[:-1]]) > 0).all() and np.bincount(ki, minlength=n).max() == 1)
    inner = np.diff(ki) > 0
    inner[off[1:-1] - 1] = True
    ok = bool(ok and inner.all())
    assert ok, "grouping differs from _.groupBy(keys, lookup)"
    del own_all, ki
    for buf in (dests, goff, kidx, owners):
        buf.free()
    stream.destroy()

    key_bytes = int(total.value)
    alg = key_bytes + 4 * args.keys + 8 * len(pts_h)  # key bytes + 4 B/key + 8 B x points
    achieved = alg / (kms / 1e3) / 1e9
    out = {
        "metric": "batched ring.lookup keys/s (config 3)",
        "value": round(args.keys / (kms / 1e3), 1),
        "unit": "keys/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": f"config 3: {args.keys} decimal u64 keys vs {args.servers} servers x 100 replicas "
                               f"({len(pts_h)} points)", "keys": args.keys, "points": int(len(pts_h)),
                   "key_bytes": key_bytes, "seed": args.seed},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": "k_lookup_keys",
                     "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(kms, 4)},
        "parity": {"sampled_keys": int(len(idx)), "mismatches": mismatches, "points_match": True},
        "group_by_owner": {"ms": round(group_ms, 3), "keys_per_s": round(n / (group_ms / 1e3), 1), "groups": g,
                           "checked": "partition by owner, input order within groups, first-appearance order"},
    }
    # SURVEY.md §8(d) ring build: 8 B x points x (read + write) x 4 radix passes
    rb_alg = 8 * len(pts_h) * 2 * 4
    rb_ms, rb_dev = min(build_ms), min(build_dev_ms)
    out["ring_build"] = {"servers": args.servers, "points": int(len(pts_h)), "ms": round(rb_ms, 3),
                         "device_ms": round(rb_dev, 3),
                         "algorithmic_bytes": rb_alg, "achieved_GBps": round(rb_alg / (rb_dev / 1e3) / 1e9, 2),
                         "frac": round(rb_alg / (rb_dev / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
                         "note": "device_ms: HIP events around rp_ring_add_remove's device work (replica hashing of "
                                 "the names copied over PCIe, 4-pass stable radix sort, dedupe, compaction, "
                                 "lookup directories); ms: host wall clock of the call; frac from device_ms"}
    if with_cpu and not args.no_cpu_baseline:
        # oracle farmhash32 (C) + numpy lower bound, one host core, on a
        # bounded sample of the same keys (strings formatted before timing)
        ks = oracle.lookup_keys(args.seed, np.arange(1_000_000))
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < min(args.cpu_seconds, 8.0):
            oracle.ring_lookup_points(oh, oo, oracle.farmhash32_batch(ks))
            done += len(ks)
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / el, 1), "unit": "keys/s", "cores": 1, "kind": "port",
                               "sample": f"oracle farmhash32 (C) + numpy lower bound over the first 1M keys, "
                                         f"{done} lookups in {el:.1f} s"}
    ring.close()
    return out


# ----------------------------------------------------------------- config 2
def run_config2(args):
    """Config 2: 1,024 nodes, ceil(1% N) = 11 re-assertions per round for 20
    rounds, then gossip until every live checksum agrees (the reference
    fixture sim_config2_n1024 converges at round 27)."""
    import ringpop_amd
    S = ringpop_amd.Sim(1024, 2024, churn_k=11)
    S.round(churn=True)  # (first-launch costs outside the clock)
    t0 = time.perf_counter()
    rounds, conv = 1, None
    while rounds < 200:
        st = S.round(churn=rounds < 20)
        rounds += 1
        if st["converged"] and rounds > 20:
            conv = rounds - 1
            break
    el = time.perf_counter() - t0
    S.close()
    return {"metric": "rounds to converge (config 2)", "value": conv, "unit": "rounds",
            "ms_per_step": round(el * 1e3 / (rounds - 1), 3),
            "config": {"workload": "config 2: 1024 nodes, 11 alive re-assertions/round for 20 rounds", "seed": 2024},
            "reference_fixture_converged_at": 27}


# ----------------------------------------------------------------- config 1
REFERENCE_JS_CONFIG1 = os.path.join(ROOT, "bench_data", "reference_js_config1.json")


def run_config1(args, iters=30):
    """Config 1 (benchmarks/large-membership-update.js:37-47,
    compute-checksum.js:46-62) on one device instance (rp_node), with the
    ready flag the published scripts forget:
      A. Membership.update() of large-membership.json's 1,332 records into a
         fresh ready instance, with the update listener's work (ring
         addRemoveServers of the alive servers, dissemination recordChange)
         and the one computeChecksum, wall clock per call from the host;
      B. computeChecksum() on 1,000 members.
    Beside it, the reference JavaScript's own time for both, measured in the
    build container (oracle/harness/time_config1.js; the reference cannot
    travel to the GPU box) and labelled as such.  Inputs are host objects
    (the drop-in's calling convention): every call includes its PCIe copies,
    launches and syncs."""
    import ringpop_amd
    recs = json.load(open(os.path.join(ROOT, "tests", "golden", "large_membership_input.json")))
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "config1_large_membership.json")))["results"]

    def instance(seed):
        node = ringpop_amd.Node("127.0.0.1:3000", rng_state=seed)
        ring = ringpop_amd.HashRing()
        diss = ringpop_amd.Dissemination(node)

        def updated(ups):  # lib/membership-update-listener.js:24-75
            add = [u["address"] for u in ups if u["status"] == "alive"]
            rm = [u["address"] for u in ups if u["status"] in ("faulty", "leave")]
            diss.recordChanges(ups)
            if (add or rm) and ring.addRemoveServers(add, rm):
                diss.adjustMaxPiggybackCount(ring.getServerCount())
        m = ringpop_amd.Membership(node, ready=True, now=lambda: 1500000000000, on_updated=updated)
        return node, ring, m

    ta = []
    for it in range(iters + 3):
        node, ring, m = instance(42 + 1332)
        batch = json.loads(json.dumps(recs))
        t0 = time.perf_counter()
        applied = m.update(batch)
        t = (time.perf_counter() - t0) * 1e3
        assert len(applied) == want["1332"]["applied"] and m.checksum == want["1332"]["checksum"]
        if it >= 3:
            ta.append(t)
        node.close()
        ring.close()
    node, ring, m = instance(42 + 1000)
    m.update(json.loads(json.dumps(recs[:1000])))
    tb = []
    for it in range(200 + 20):
        t0 = time.perf_counter()
        cs = m.computeChecksum()
        if it >= 20:
            tb.append((time.perf_counter() - t0) * 1e3)
    assert cs == want["1000"]["checksum"]
    node.close()
    ring.close()
    med = lambda a: sorted(a)[len(a) // 2]  # noqa: E731
    out = {"metric": "config 1 latency (one instance, host objects in and out)", "unit": "ms",
           "update_1332": {"median_ms": round(med(ta), 3), "min_ms": round(min(ta), 3), "iterations": len(ta),
                           "checked": "applied count and checksum equal the reference fixture"},
           "compute_checksum_1000": {"median_ms": round(med(tb), 4), "min_ms": round(min(tb), 4),
                                     "iterations": len(tb), "checked": "checksum equals the reference fixture"}}
    if os.path.exists(REFERENCE_JS_CONFIG1):
        js = json.load(open(REFERENCE_JS_CONFIG1))
        out["reference_js"] = {
            "measured": "in the build container (node " + js["node"] + ", one core, farmhash = the harness's JS "
                        "transcription), not on the GPU box: oracle/harness/time_config1.js",
            "update_1332_median_ms": round(js["update_1332"]["median_ms"], 3),
            "compute_checksum_1000_median_ms": round(js["compute_checksum_1000"]["median_ms"], 4)}
    return out


# ----------------------------------------------------------------- config 5
def run_failure(args, world=1, rank=0, dist=None, sim_cls=None):
    """Config 5: fail-stop ceil(fail_frac * N) seeded nodes at round 0, plus a
    seeded false-suspicion storm (--storm-ppm of the live nodes per round for
    --storm-rounds rounds: makeSuspect by a live accuser, refuted by the
    victim), and gossip (ping, ping-req relays, suspicion timers -> faulty)
    until every live view is identical with every failed node faulty.
    Reports rounds-to-converge; member-updates/s over the run.  No churn
    unless --churn is given.  N > 1 ranks (or --shards): the cluster is
    sharded exactly as config 4, the ping-req waves cross shards over RCCL."""
    import numpy as np

    n = args.nodes
    k = args.churn if args.churn is not None else 0
    nf = math.ceil(args.fail_frac * n)
    dead = np.sort(np.random.default_rng(args.seed).choice(n, size=nf, replace=False)).tolist()
    storm = {"start": 0, "end": args.storm_rounds, "ppm": args.storm_ppm} if args.storm_ppm else None
    live = np.ones(n, dtype=bool)
    live[dead] = False

    def converge(S, lo, hi):
        rounds, converged_at, first_agree, last = 0, None, None, time.perf_counter()
        while rounds < args.max_rounds:
            st = S.round(churn=k > 0)  # counters and the convergence flag are cluster-wide
            rounds += 1
            if rank == 0 and time.perf_counter() - last > 20:
                print(f"round {rounds}: evaluated {st['evaluated']} applied {st['applied']} "
                      f"full_syncs {st['full_syncs']} waves {st['waves']}", file=sys.stderr, flush=True)
                last = time.perf_counter()
            if st["converged"] and rounds > args.storm_rounds:
                first_agree = first_agree or rounds
                # converged for good: every failed node faulty in every live view
                vc = S.view_counts()[lo:hi][live[lo:hi]]
                done = bool((vc[:, 3] == nf).all())
                if dist:
                    import torch
                    t = torch.tensor([1 if done else 0], dtype=torch.int32)
                    dist.all_reduce(t, op=dist.ReduceOp.MIN)
                    done = bool(t.item())
                if done:
                    converged_at = rounds
                    break
        S.sync()
        return rounds, converged_at, first_agree

    # One process, one shard: the run the line's time is quoted on carries no
    # per-stage HIP events (two per stage launch on the round's stream); the
    # same seeded run is repeated with them for kernel_ms and the checksum
    # split (it must converge in the same round: the simulation is deterministic).
    clean = None
    if world == 1 and args.shards <= 1 and sim_cls is None:
        S, mode, _ = make_sim(args, n, k, world, rank, dist, sim_cls=sim_cls, failures={0: dead}, storm=storm)
        lo, hi = S.shard_range()
        S.sync()
        t0 = time.perf_counter()
        clean = converge(S, lo, hi)
        clean = clean + (time.perf_counter() - t0,)
        S.close()
    S, mode, _ = make_sim(args, n, k, world, rank, dist, sim_cls=sim_cls, failures={0: dead}, storm=storm)
    lo, hi = S.shard_range()
    S.sync()
    c0 = S.counters()
    S.enable_timing(True)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    rounds, converged_at, first_agree = converge(S, lo, hi)
    elapsed = time.perf_counter() - t0
    elapsed_timed = elapsed
    if clean is not None:
        if clean[:3] != (rounds, converged_at, first_agree):
            raise RuntimeError(f"config 5 not deterministic: {clean[:3]} vs {(rounds, converged_at, first_agree)}")
        elapsed = clean[3]
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    c1 = S.counters()
    kt = S.kernel_times()
    mem_used = None
    try:
        from ringpop_amd import hiprt
        free_b, total_b = hiprt.memory()
        mem_used = round((total_b - free_b) / 1e9, 1)
    except Exception:  # noqa: BLE001 - (host-only tests run a stand-in simulation)
        pass
    d = {key: c1[key] - c0[key] for key in c1}
    vc = S.view_counts()[lo:hi][live[lo:hi]]
    cs = S.checksums()[lo:hi]
    out = {
        "metric": "rounds to converge after a 10% mass failure + false-suspicion storm (config 5)",
        "value": converged_at,
        "unit": "rounds",
        "n_gpus": world, "steps": rounds, "warmup": 0,
        "ms_per_step": round(elapsed * 1e3 / rounds, 3),
        "ms_per_step_with_stage_events": round(elapsed_timed * 1e3 / rounds, 3),
        "higher_is_better": False, "scaling": "strong",  # one fixed cluster at every N
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": f"config 5: {n} nodes, {nf} fail-stopped at round 0, 25-round suspicion timeout, "
                               f"false-suspicion storm {args.storm_ppm} ppm of live nodes/round for "
                               f"{args.storm_rounds} rounds", "nodes": n, "failed": nf, "churn_per_round": k,
                   "storm": storm, "seed": args.seed, "parallelism": mode},
        "first_agreement_round": first_agree,
        "member_updates_per_s": round(d["evaluated"] / elapsed, 1),
        "applied": d["applied"], "full_syncs": d["full_syncs"], "messages": d["messages"],
        "end_state": {"live_checksums_distinct": int(len(np.unique(cs[live[lo:hi]]))),
                      "live_views_checked": int(len(vc)),
                      "every_failed_faulty": bool((vc[:, 3] == nf).all()),
                      "no_suspects_left": bool((vc[:, 2] == 0).all()),
                      "every_ring_holds_live_servers": bool((vc[:, 5] == n - nf).all())},
        "kernel_ms": {c: round(v[0], 3) for c, v in kt.items()},
        "device_memory_used_gb": mem_used,
    }
    # the checksum stage (predicate, fingerprint dedupe and cache, k_checksums
    # with one wave rendering and hashing one view, k_pending): algorithmic
    # bytes = the view cells read, 16 B x n per view hashed;
    # a k_checksums launch is bounded by its longest sequential farmhash
    # chain (one 2.3 MB string per view at 65,536 nodes), not by HBM
    ck_ms, ck_launches = kt.get("checksum", (0.0, 0))
    # one shard: the chains run on a side stream beside the merges (rp_sim_side_ms);
    # "ms" is the checksum time left on the round's own stream (exposed)
    side = S.side_ms() if hasattr(S, "side_ms") else 0.0
    views = d.get("checksum_views", 0)
    if ck_launches and views:
        ck_bytes = 16.0 * n * views
        tot = ck_ms + side
        out["checksum"] = {"views_hashed": views, "stages": ck_launches, "ms": round(ck_ms, 3),
                           "exposed_ms": round(ck_ms, 3), "side_stream_ms": round(side, 3),
                           "total_ms": round(tot, 3),
                           "note": "exposed: on the round's stream; side_stream: the sender checksum chains and "
                                   "fullSync decisions on a second stream beside the ping and response merges",
                           "roofline": {"bound": "latency (sequential farmhash chain per view)",
                                        "achieved": round(ck_bytes / (tot / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                                        "unit": "GB/s", "frac": round(ck_bytes / (tot / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                        "algorithmic_bytes_per_view": 16 * n}}
    if world > 1 or args.shards > 1:
        out["exchange"] = exchange_report(S.exchange_stats(), rank, world, kt, dist)
    S.close()
    return out


def exchange_report(xs, rank, world, kt, dist):
    """Exchange traffic per rank: with one process per GPU each rank reports
    the bytes it sent (all-gathers, all-to-alls, all-reduces); in-process
    shards report each shard's outgoing device copies as its rank's.  Every
    rank's list is gathered to rank 0 (a collective: every rank calls this)."""
    rounds = max(xs["rounds"], 1)
    sb = xs.get("shard_bytes") or [xs["bytes_sent"]]
    km = {c: round(v[0], 3) for c, v in kt.items()}
    if dist:
        mine = [{"rank": rank, "bytes_sent": sb[0], "bytes_sent_per_round": round(sb[0] / rounds),
                 "exchange_ms": round(xs["ms"], 3), "kernel_ms": km}]
        allr = [None] * world
        dist.all_gather_object(allr, mine[0])
        ranks = allr
    else:  # in-process shards: one stream and one host thread each, timing on shard 0's stream
        ranks = [{"rank": i, "bytes_sent": b, "bytes_sent_per_round": round(b / rounds)} for i, b in enumerate(sb)]
        ranks[0].update({"exchange_ms": round(xs["ms"], 3), "kernel_ms": km})
    per_round = [r["bytes_sent_per_round"] for r in ranks]
    return {"ms": round(xs["ms"], 3), "rounds": xs["rounds"],
            "bytes_sent_rank0": ranks[0]["bytes_sent"], "bytes_per_round_rank0": per_round[0],
            "bytes_per_round_max_rank": max(per_round), "bytes_per_round_all_ranks": sum(per_round),
            "alltoall_bytes_all_ranks": xs["bytes_sent"] if not dist else None,
            "per_rank": ranks}


def run_loop_ranks(args):
    """--loop-ranks G (one GPU): the config-4 or config-5 cluster as G ranks of
    the one-process-per-GPU code (rp_sim_create_rank's plans, counts and
    buffers), each driven by its own host thread, the collectives device
    copies after a rendezvous of the threads (the loopback transport).  The
    ranks share one GPU, so this measures the rank path's host structure and
    exchange volume, not multi-GPU scaling."""
    import threading

    import numpy as np

    import ringpop_amd
    from ringpop_amd.sim import Loop
    G, n = args.loop_ranks, args.nodes
    fail = args.workload == "failure"
    k = args.churn if args.churn is not None else (0 if fail else math.ceil(0.01 * n))
    kw = {"churn_k": k}
    if fail:
        nf = math.ceil(args.fail_frac * n)
        dead = np.sort(np.random.default_rng(args.seed).choice(n, size=nf, replace=False)).tolist()
        kw["failures"] = {0: dead}
        kw["arena_entries"] = (n // G) * 32768
        if args.storm_ppm:
            kw["storm"] = {"start": 0, "end": args.storm_rounds, "ppm": args.storm_ppm}
    loop = Loop(G)
    sims = [ringpop_amd.Sim(n, args.seed, shards=G, rank=r, loop=loop, **kw) for r in range(G)]
    errs = [None] * G

    def par(fn):
        def body(r):
            try:
                fn(r, sims[r])
            except Exception as e:  # noqa: BLE001 - raised below for all ranks
                errs[r] = repr(e)
        th = [threading.Thread(target=body, args=(r,)) for r in range(G)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if any(errs):
            raise RuntimeError("loop ranks failed: %s" % errs)

    out = {"n_gpus": 1, "higher_is_better": not fail, "vs_baseline": None, "dtype": "u64", "data": "synthetic"}
    if not fail:
        par(lambda r, S: (S.run(args.preroll + args.warmup, churn=True), S.sync()))
        c0 = sims[0].counters()
        par(lambda r, S: S.enable_timing(True))
        t0 = time.perf_counter()
        par(lambda r, S: (S.run(args.steps, churn=True), S.sync()))
        elapsed = time.perf_counter() - t0
        d = {key: v - c0[key] for key, v in sims[0].counters().items()}
        steps = args.steps
        out.update({"metric": METRIC, "value": round(d["evaluated"] / elapsed, 1), "unit": "member-updates/s",
                    "steps": steps, "warmup": args.warmup, "scaling": "strong",
                    "rounds_per_s": round(steps / elapsed, 3)})
        workload = f"config 4: {n} simulated ringpop nodes, {k} alive re-assertions/round, after a {args.preroll}-round pre-roll"
    else:
        live = np.ones(n, dtype=bool)
        live[dead] = False
        bar = threading.Barrier(G)
        votes, result = [False] * G, {}

        def rounds_until_converged(r, S):
            S.enable_timing(True)
            lo, hi = S.shard_range()
            for rr in range(1, args.max_rounds + 1):
                st = S.round(churn=k > 0)
                ok = bool(st["converged"]) and rr > args.storm_rounds
                if ok:
                    vc = S.view_counts()[lo:hi][live[lo:hi]]
                    ok = bool((vc[:, 3] == nf).all())
                votes[r] = ok
                bar.wait()
                stop = all(votes)
                bar.wait()
                if stop:
                    result[r] = rr
                    return
            result[r] = None
        t0 = time.perf_counter()
        par(rounds_until_converged)
        elapsed = time.perf_counter() - t0
        steps = result[0] or args.max_rounds
        out.update({"metric": "rounds to converge after a 10% mass failure + false-suspicion storm (config 5)",
                    "value": result[0], "unit": "rounds", "steps": steps, "warmup": 0, "scaling": "strong"})
        workload = (f"config 5: {n} nodes, {nf} fail-stopped at round 0, false-suspicion storm "
                    f"{args.storm_ppm} ppm for {args.storm_rounds} rounds")
    per_rank = []
    for r, S in enumerate(sims):
        xs = S.exchange_stats()
        b = (xs.get("shard_bytes") or [xs["bytes_sent"]])[0]
        kt = S.kernel_times()
        rounds = max(xs["rounds"], 1)
        # (device time of this rank's own kernels on its stream, per round:
        # with all ranks on one GPU they also slow each other down)
        per_rank.append({"rank": r, "bytes_sent": b, "bytes_sent_per_round": round(b / rounds),
                         "kernel_ms_per_round": {c: round(v[0] / rounds, 4) for c, v in kt.items()},
                         "exchange_ms_per_round": round(xs["ms"] / rounds, 4)})
    out["ms_per_step"] = round(elapsed * 1e3 / steps, 3)
    out["config"] = {"workload": workload, "nodes": n, "seed": args.seed, "parallelism": f"loop-ranks{G}"}
    out["exchange"] = {"bytes_per_round_max_rank": max(x["bytes_sent_per_round"] for x in per_rank),
                       "per_rank": per_rank}
    for S in sims:
        S.close()
    loop.close()
    return out


class ShardBuildError(RuntimeError):
    """A rank of a multi-GPU run could not build its shard of the cluster."""


def make_sim(args, n, k, world, rank, dist, sim_cls=None, failures=None, storm=None):
    """This rank's simulation.  N > 1: one shard of the 65,536-node cluster per
    GPU, exchanging over RCCL inside libringpop_hip (the communicator id is
    broadcast over the gloo group).  If any rank cannot build its shard, every
    rank raises ShardBuildError together (the errors are all-gathered first, so
    no rank is left waiting in a collective): a multi-GPU line is the sharded
    cluster or nothing -- never N independent replicas summed.
    Returns (sim, parallelism label, None)."""
    if sim_cls is None:
        import ringpop_amd
        sim_cls = ringpop_amd.Sim
    kw = {"churn_k": k, "failures": failures}
    if storm:
        kw["storm"] = storm
    G = world if world > 1 else max(args.shards, 1)
    if failures and G > 1:
        # a shard's message arena sized for config 5's logs (an issue reserves
        # room for every live key, and every faulty and suspect update stays
        # live for maxPiggybackCount issues): 2x the default
        kw["arena_entries"] = (n // G) * 32768
    if world == 1 and args.shards <= 1:
        return sim_cls(n, args.seed, **kw), "single", None
    if world == 1:
        return sim_cls(n, args.seed, shards=args.shards, **kw), f"shards{args.shards}-in-process", None
    obj = [sim_cls.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    S, err = None, None
    try:
        S = sim_cls(n, args.seed, shards=world, rank=rank, unique_id=obj[0], **kw)
    except Exception as e:  # noqa: BLE001 - every rank learns of it below
        err = f"rank {rank}: {e}"
    errs = [None] * world
    dist.all_gather_object(errs, err)
    errs = [e for e in errs if e]
    if not errs:
        return S, f"sharded{world}-rccl", None
    if S is not None:
        S.close()
    raise ShardBuildError("; ".join(errs)[:500])


# ----------------------------------------------------------------- config 4 (headline)
def run_gossip(args, world, rank, dist, sim_cls=None):
    n = args.nodes
    k = args.churn if args.churn is not None else math.ceil(0.01 * n)
    # this box's ceilings and clocks (the real device only; every rank measures its own GPU)
    # (RP_BENCH_NO_CAL=1: skip it -- experiments on the allocation order only)
    box = box_ceiling() if sim_cls is None and not os.environ.get("RP_BENCH_NO_CAL") else None
    clk = ClockSampler(_pci_bus_id()) if sim_cls is None else None
    S, mode, _ = make_sim(args, n, k, world, rank, dist, sim_cls=sim_cls)
    # pre-roll to the steady state the line is quoted on (the log fill of a
    # node takes ~50 rounds to stop growing), then the warmup rounds
    S.run(args.preroll + args.warmup, churn=True)
    S.sync()
    c0, l0 = S.counters(), S.local_counters()

    def barrier():
        S.sync()  # device work of this rank drained (the sim's own stream)
        if dist:
            dist.barrier()

    # Only the line's roofline stage (the ping merge) carries HIP events inside
    # the timed region -- two per stage launch on the simulation stream, ~0.1
    # ms per round when every stage has them -- and a second pass of the same
    # length right after times every stage (and the exchange steps) for the
    # per-stage breakdown and the exchange report.
    S.enable_timing(True, stages=["merge_ping"])
    barrier()
    if clk:
        clk.start()  # (a host thread reading sysfs: no HIP call)
    t0 = time.perf_counter()
    S.run(args.steps, churn=True)
    S.sync()
    t1 = time.perf_counter()
    if clk:
        clk.stop()
    barrier()
    elapsed = t1 - t0
    c1, l1 = S.counters(), S.local_counters()
    kt_timed = S.kernel_times()
    d = {key: c1[key] - c0[key] for key in c1}
    dl_timed = {key: l1[key] - l0[key] for key in l1}
    S.enable_timing(True)
    S.run(args.steps, churn=True)
    S.sync()
    l2 = S.local_counters()
    kt = S.kernel_times()
    xs = S.exchange_stats()
    dl = {key: l2[key] - l1[key] for key in l2}

    # (the sharded counters are cluster-wide already: no sum over ranks)
    tot = {key: float(d[key]) for key in ("evaluated", "applied", "touched")}
    if dist:
        import torch
        mx = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed = float(mx[0].item())

    # per rank (or in-process shard): its exchange traffic, and its kernel time per stage
    xrep = exchange_report(xs, rank, world, kt, dist) if (world > 1 or args.shards > 1) else None

    observed = None
    if world == 1 and args.shards <= 1 and not args.no_extras:
        # tick-cluster's convergence check (scripts/tick-cluster.js:88-115):
        # every live node's membership checksum read after every round.  The
        # device computes farmhash checksums when read; here all
        # of them are, every round (views that differ hash separately)
        S.round(churn=True)  # (untimed: the first launch of the many-view checksum kernel loads its code)
        S.checksums()
        S.sync()
        t0o = time.perf_counter()
        nobs = 3
        ck_s = 0.0
        for _ in range(nobs):
            S.round(churn=True)
            S.sync()
            t1o = time.perf_counter()
            S.checksums()  # (synchronous: the checksums are on the host when it returns)
            ck_s += time.perf_counter() - t1o
        el_o = time.perf_counter() - t0o
        observed = {"rounds_per_s": round(nobs / el_o, 3), "ms_per_round": round(el_o * 1e3 / nobs, 3),
                    "checksums_ms": round(ck_s * 1e3 / nobs, 3),
                    "rounds": nobs, "note": "each round followed by every node's farmhash checksum "
                                            "(rp_sim_read_checksums: all 65,536 views rendered and hashed, "
                                            "deduplicated by content fingerprint), read back to the host"}

    if rank != 0:
        S.close()
        return None

    # Stages of a round on this rank (own shard's counters, HIP-event device
    # time on the simulation stream): the ping merge (merge + issueAsReceiver
    # per ping: k_p2_lists, k_p2_apply x2, k_p2_respond x2, k_phase2), the
    # response merge (k_phase3) and the sender issue (k_iterate, k_shuffle,
    # k_phase1).  One definition for all: work bytes / device time.
    def stage(cat, touched, applied, scanned, written, ev, kernel, kt=kt):
        ms, launches = kt[cat]
        per_s = (ms / 1000.0) / max(launches, 1)
        work = (WORK_B_TOUCHED * touched + WORK_B_APPLIED * applied + WORK_B_SCANNED * scanned
                + WORK_B_WRITTEN * written) / max(launches, 1)
        ach = work / per_s / 1e9 if per_s > 0 else 0.0
        o = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kernel,
             "work_bytes_per_launch": int(work), "avg_launch_ms": round(per_s * 1e3, 4), "launches": launches,
             "units_per_launch": {k: int(v / max(launches, 1)) for k, v in
                                  (("touched", touched), ("applied", applied), ("log_words_scanned", scanned),
                                   ("written", written))}}
        if applied:
            # the merge against its own access ceiling: applied changes (each a
            # random view-cell read-modify-write) per second
            ach = applied / max(launches, 1) / per_s if per_s > 0 else 0.0
            o["random_rmw"] = {"achieved_per_s": round(ach, 1), "peak_per_s": RANDOM_RMW_PEAK,
                               "frac": round(ach / RANDOM_RMW_PEAK, 4),
                               "note": "applied changes / stage time vs the measured random 16-B cell "
                                       "read-modify-write rate (tools/micro/fetch_cal.hip)"}
        if ev is not None:
            ref = (MERGE_B_EVAL * ev + MERGE_B_APPLIED * applied) / max(launches, 1)
            o["reference_equivalent"] = {
                "bytes_per_launch": int(ref), "GBps": round(ref / per_s / 1e9, 2) if per_s > 0 else 0.0,
                "note": "SURVEY §8(d): 32 B x the reference's evaluated list entries + 32 B x applied; most "
                        "evaluated entries are provable no-ops the sender leaves out (seen filter), so this can "
                        "exceed the bytes moved"}
        return o

    stages = {
        "ping_merge": stage("merge_ping", dl["touched_ping_merge"], dl["applied_ping_merge"], dl["scanned_recv_issue"],
                            dl["written_recv_issue"], dl["eval_ping_merge"],
                            "k_phase2 stage (k_p2_lists, k_p2_apply x2, k_p2_respond x2, k_phase2)"),
        "resp_merge": stage("merge_resp", dl["touched"] - dl["touched_ping_merge"], dl["applied_resp_merge"], 0, 0,
                            dl["eval_resp_merge"], "k_phase3"),
        "send_issue": stage("issue", 0, 0, dl["scanned_send_issue"], dl["written_send_issue"], None,
                            "issue stage (k_iterate, k_shuffle, k_phase1)"),
    }
    # the line's roofline: the stage with the most device time (the ping merge in steady state)
    name = max(stages, key=lambda c: stages[c]["avg_launch_ms"] * stages[c]["launches"])
    roofline = dict(stages[name])
    roofline["stage"] = name
    if name == "ping_merge":
        # its launches timed inside the timed region itself (the only stage with events there)
        roofline = stage("merge_ping", dl_timed["touched_ping_merge"], dl_timed["applied_ping_merge"],
                         dl_timed["scanned_recv_issue"], dl_timed["written_recv_issue"], dl_timed["eval_ping_merge"],
                         "k_phase2 stage (k_p2_lists, k_p2_apply x2, k_p2_respond x2, k_phase2)", kt=kt_timed)
        roofline["stage"] = name
        roofline["timing"] = ("HIP events around this stage's launches on the simulation stream, inside the "
                              "timed region; the other stages and kernel_ms from a second pass of --steps rounds")
    if box:
        for st in stages.values():
            st["frac_of_box"] = frac_of_box(st, box)
        roofline["frac_of_box"] = frac_of_box(roofline, box)

    value = tot["evaluated"] / elapsed
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "member-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True,
        # the 65,536-node cluster is one fixed job at every N (N = 1 included)
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"config 4: {n} simulated ringpop nodes, full views, {k} alive re-assertions/round, "
                               f"timed after a {args.preroll}-round pre-roll + {args.warmup} warmup rounds "
                               "(steady-state log fill)",
                   "nodes": n, "churn_per_round": k, "seed": args.seed, "preroll": args.preroll,
                   "parallelism": mode},
        "rounds_per_s": round(args.steps / elapsed, 3),
        "applied_per_s": round(tot["applied"] / elapsed, 1),
        # the reference's accounting counts every change in every list; the
        # seen filter leaves provable no-ops out of messages, so only these
        # were physically evaluated against a view cell
        "touched_per_s": round(tot["touched"] / elapsed, 1),
        "seen_filter_fraction": round(1.0 - tot["touched"] / max(tot["evaluated"], 1.0), 4),
        "evaluated_per_round": round(tot["evaluated"] / args.steps, 1),
        "kernel_ms": {c: round(v[0], 3) for c, v in kt.items()},
        "roofline": roofline,
        "stages": stages,
    }
    if box:
        out["box_ceiling"] = box
    if clk:
        out["clocks"] = clk.report()
    if observed:
        out["observed_checksums"] = observed
    if xrep:
        out["exchange"] = xrep
    S.close()
    return out


def _sub(line, keys):
    return {k: line[k] for k in keys if k in line}


def visible_gpus():
    """GPUs the rank processes could use, counted without the HIP runtime (the
    launcher parent must not start it before spawning its ranks): the
    *_VISIBLE_DEVICES lists when set, else the KFD topology's GPU nodes
    (gpu_id != 0; CPU nodes have 0)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val is not None:
            return len([x for x in val.split(",") if x.strip() and x.strip() != "-1"])
    root = "/sys/class/kfd/kfd/topology/nodes"
    count = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "gpu_id")) as f:
                    count += int(f.read().strip() or "0") != 0
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    return count


def launch_ranks(args, argv, child=None, devices=None, timeout_s=3600):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the
    environment): start N fresh rank processes of this script, one per GPU,
    exactly as `torch.distributed.run --nproc-per-node N` would (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), and
    pass rank 0's JSON line through.  The parent never touches the GPU and
    never execs; if any rank fails, the others are stopped (by their own
    process handles) and the parent exits with that rank's status.
    `child` / `devices` replace the rank command and the device count (CPU
    tests)."""
    import socket
    import subprocess
    n = args.gpus
    have = visible_gpus() if devices is None else devices
    if have < n:
        print(f"bench.py --gpus {n}: only {have} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = child or [sys.executable, "-u", os.path.abspath(__file__)] + list(argv)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    # rank 0's stdout is read on a thread (a full pipe would block the rank)
    got = []
    import threading
    reader = threading.Thread(target=lambda: got.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    t0, rc = time.time(), 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad or time.time() - t0 > timeout_s:
            rc = bad[0] if bad else 124
            rc = 128 - rc if rc < 0 else rc  # (killed by a signal)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    reader.join(timeout=30)
    if got and got[0]:
        sys.stdout.write(got[0].decode())
        sys.stdout.flush()
    return rc


def main(argv=None, sim_cls=None):
    """sim_cls: a stand-in for ringpop_amd.Sim (CPU tests of the multi-rank
    host logic): no library build and no device selection then."""
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        print(f"bench.py --gpus {args.gpus} under a launcher of {world} ranks", file=sys.stderr, flush=True)
        return 2
    if args.workload == "lookup":
        print(json.dumps(run_lookup(args)), flush=True)
        return 0
    traffic = None
    if (world == 1 and args.shards <= 1 and args.loop_ranks <= 1 and args.workload == "gossip" and sim_cls is None
            and not args.no_traffic):
        # (child runs under rocprofv3 before this process touches the GPU:
        # two 65,536-node clusters do not fit in HBM together)
        try:
            traffic = pmc_traffic(args)
        except Exception as e:  # noqa: BLE001 - reported in the line, never fatal
            traffic = {"error": repr(e)[:400]}
        if not args.no_extras:
            try:
                traffic["lookup"] = lookup_pmc(args)
            except Exception as e:  # noqa: BLE001
                traffic["lookup"] = {"error": repr(e)[:400]}
    dist = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        # host-side coordination only (barriers, the RCCL id, result
        # reductions); the data path is RCCL inside libringpop_hip
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=15))

    if sim_cls is None:
        from ringpop_amd import build
        from ringpop_amd._lib import check, lib
        if rank == 0 or world == 1:
            build.build()
        if dist:
            dist.barrier()
        check(lib().rp_set_device(local))
    elif dist:
        dist.barrier()
    if args.loop_ranks > 1 and world == 1:
        print(json.dumps(run_loop_ranks(args)), flush=True)
        return 0
    try:
        if args.workload == "failure":
            out = run_failure(args, world, rank, dist, sim_cls=sim_cls)
            if rank == 0:
                print(json.dumps(out), flush=True)
            if dist:
                dist.destroy_process_group()
            return 0
        out = run_gossip(args, world, rank, dist, sim_cls=sim_cls)
    except ShardBuildError as e:
        # no number without the sharded cluster: a null line naming the error, and a failing status
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "member-updates/s", "n_gpus": world,
                              "error": "sharded cluster unavailable: " + str(e)}), flush=True)
        print(f"bench.py rank {rank}: sharded cluster unavailable: {e}", file=sys.stderr, flush=True)
        if dist:
            dist.destroy_process_group()
        return 3
    if out is not None and traffic is not None:
        attach_traffic(out, traffic)
    if out is not None and world == 1 and args.shards <= 1:
        if not args.no_extras:
            # configs 3 and 5 on the same GPU, after the headline cluster is freed
            sub = argparse.Namespace(**vars(args))
            sub.steps, sub.warmup = 10, 2
            lk = run_lookup(sub, with_cpu=not args.no_cpu_baseline)
            out["config3"] = _sub(lk, ("metric", "value", "unit", "ms_per_step", "config", "roofline", "parity",
                                       "group_by_owner", "ring_build", "cpu_baseline"))
            lp = (traffic or {}).get("lookup")
            if lp and "traffic" in lp:
                r3 = out["config3"]["roofline"]
                r3["traffic"] = lp["traffic"]
                r3["traffic_frac"] = round(lp["traffic"] / (r3["avg_launch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                r3["l2_misses_per_key"] = lp["l2_misses_per_key"]
                r3["l2_hits_per_key"] = lp["l2_hits_per_key"]
                # the directory (4 MB) and points (8 MB) live in the 256 MB
                # Infinity Cache, which FETCH_SIZE counts too: the random
                # lines of L2 misses bound it, not HBM streaming
                r3["bound"] = "l2-miss latency (random directory / point lines, Infinity-Cache resident)"
                r3["pmc"] = lp["method"]
            elif lp:
                out["config3"]["roofline"]["pmc_error"] = lp.get("error")
            out["config2"] = run_config2(args)
            out["config1"] = run_config1(args)
            fl = run_failure(args)
            out["config5"] = _sub(fl, ("metric", "value", "unit", "steps", "ms_per_step",
                                       "ms_per_step_with_stage_events", "config",
                                       "first_agreement_round", "member_updates_per_s", "full_syncs", "end_state",
                                       "kernel_ms", "checksum"))
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, out["evaluated_per_round"])
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
