"""bench.py --gpus N started without torchrun (CPU, gloo): the parent starts N
rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in each
child's environment, no exec, no GPU call in the parent) and passes rank 0's
JSON line through.  The ranks build a stand-in simulation (FakeGossipSim)
through bench.main(sim_cls=...), so the whole multi-rank host path -- the RCCL
id broadcast, the barrier-bracketed timed region, the max over ranks, the
per-rank exchange report -- runs here without a device."""
import json
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

STAGE_KEYS = ("touched_ping_merge", "applied_ping_merge", "scanned_recv_issue", "written_recv_issue",
              "eval_ping_merge", "touched", "applied_resp_merge", "eval_resp_merge", "scanned_send_issue",
              "written_send_issue")


class FakeGossipSim:
    """Stands in for one rank's shard of ringpop_amd.Sim (config 4)."""

    def __init__(self, n, seed, churn_k=None, shards=1, rank=None, unique_id=None, failures=None, storm=None,
                 arena_entries=0):
        if rank is not None and str(rank) == os.environ.get("FAKE_FAIL_RANK"):
            raise RuntimeError("ncclCommInitRank: unhandled system error")
        self.n, self.shards, self.rank, self.uid, self.r = n, shards, rank, unique_id, 0
        self.log = []

    @staticmethod
    def unique_id():
        return b"\x05" * 128

    def run(self, k, churn=True):
        self.r += k

    def sync(self):
        pass

    def enable_timing(self, on, stages=None):
        self.log.append(("timing", on, stages))

    def counters(self):  # cluster-wide counters (every rank sees the same)
        return {"evaluated": 1000 * self.r, "applied": 10 * self.r, "touched": 20 * self.r}

    def local_counters(self):
        return {k: 5 * self.r for k in STAGE_KEYS}

    def kernel_times(self):
        return {"merge_ping": (2.0, 4), "merge_resp": (1.0, 4), "issue": (1.0, 4)}

    def exchange_stats(self):
        return {"ms": 1.5, "bytes_sent": 4096 * ((self.rank or 0) + 1) * self.r, "rounds": self.r}

    def close(self):
        pass


CHILD = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); import bench, test_bench_launcher as t; "
         "sys.exit(bench.main(sys.argv[1:], sim_cls=t.FakeGossipSim))")


def _run(n, extra=(), fail_rank=None):
    argv = ["--gpus", str(n), "--steps", "3", "--warmup", "1", "--preroll", "2", "--nodes", "64", *extra]
    child = [sys.executable, "-c", CHILD % (ROOT, os.path.join(ROOT, "tests"))] + argv
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FAKE_FAIL_RANK")}
    if fail_rank is not None:
        env["FAKE_FAIL_RANK"] = str(fail_rank)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "a = bench.parse(%r); sys.exit(bench.launch_ranks(a, %r, child=%r, devices=%d))"
            % (ROOT, argv, argv, child, n))
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)


def test_gpus2_without_torchrun_launches_two_ranks():
    p = _run(2)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "sharded2-rccl"
    assert out["steps"] == 3 and out["scaling"] == "strong" and "fallback" not in out
    ranks = out["exchange"]["per_rank"]
    assert [r["rank"] for r in ranks] == [0, 1]
    assert ranks[1]["bytes_sent"] == 2 * ranks[0]["bytes_sent"] > 0  # each rank reports its own


def test_launcher_refuses_more_ranks_than_gpus():
    args = bench.parse(["--gpus", "4"])
    assert bench.launch_ranks(args, ["--gpus", "4"], child=[sys.executable, "-c", "pass"], devices=1) == 2


def test_launcher_stops_the_other_ranks_when_one_fails():
    """A rank that dies takes the job down with its status instead of leaving
    the others waiting in a collective."""
    child = [sys.executable, "-c", "import os, sys, time; r = int(os.environ['RANK']); "
             "sys.exit(3) if r == 1 else time.sleep(120)"]
    args = bench.parse(["--gpus", "2"])
    import time
    t0 = time.time()
    assert bench.launch_ranks(args, [], child=child, devices=2) == 3
    assert time.time() - t0 < 60


def test_gpus2_shard_failure_is_loud():
    """A rank that cannot build its shard (an RCCL init failure, say) makes the
    whole job fail: a non-zero status and a line with value null naming the
    error -- never the sum of independent replicas."""
    p = _run(2, fail_rank=1)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["value"] is None and out["n_gpus"] == 2
    assert "rank 1" in out["error"] and "ncclCommInitRank" in out["error"]


def test_visible_gpus_does_not_start_hip():
    """The launcher parent counts GPUs without torch or HIP: after
    visible_gpus() the process has not even imported torch."""
    code = ("import sys; sys.path.insert(0, %r); import bench; n = bench.visible_gpus(); "
            "assert isinstance(n, int) and n >= 0; assert 'torch' not in sys.modules, 'torch imported'; "
            "import os; os.environ['HIP_VISIBLE_DEVICES'] = '0,1,2'; assert bench.visible_gpus() == 3" % ROOT)
    env = {k: v for k, v in os.environ.items() if not k.endswith("_VISIBLE_DEVICES")}
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]


def test_single_gpu_times_only_the_ping_merge_inside_the_timed_region():
    """One process: the timed rounds carry HIP events for the roofline stage
    only; a second pass of --steps rounds times every stage for the breakdown."""
    args = bench.parse(["--steps", "3", "--warmup", "1", "--preroll", "2", "--nodes", "64", "--no-extras",
                        "--no-cpu-baseline", "--no-traffic"])
    made = []

    class Recorder(FakeGossipSim):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            made.append(self)

    out = bench.run_gossip(args, 1, 0, None, sim_cls=Recorder)
    (S,) = made
    timing = [e for e in S.log if e[0] == "timing"]
    assert timing == [("timing", True, ["merge_ping"]), ("timing", True, None)]
    assert S.r == 2 + 1 + 3 + 3  # pre-roll + warmup, the timed rounds, the per-stage pass
    assert out["roofline"]["stage"] == "ping_merge" and "timing" in out["roofline"]
    assert out["ms_per_step"] >= 0 and out["steps"] == 3
