"""World-size-2 gloo tests (CPU) of bench.py's multi-GPU host logic: the RCCL
communicator id is broadcast from rank 0, every rank builds its shard, and if
any rank cannot, all ranks raise ShardBuildError together (no rank is left
waiting in a collective, and no replica sum is ever reported)."""
import os
import socket
import sys
import types

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeSim:
    """Stands in for ringpop_amd.Sim (no GPU here): records how it was built."""
    fail_rank = None

    def __init__(self, n, seed, churn_k=None, shards=1, rank=None, unique_id=None, failures=None):
        if rank is not None and rank == FakeSim.fail_rank:
            raise RuntimeError("no device")
        self.args = (n, seed, churn_k, shards, rank, unique_id)
        self.closed = False

    @staticmethod
    def unique_id():
        return b"\x07" * 128

    def close(self):
        self.closed = True


def _worker(rank, world, port, fail_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    FakeSim.fail_rank = fail_rank
    args = types.SimpleNamespace(seed=10, shards=1)
    try:
        S, mode, fallback = bench.make_sim(args, 64, 1, world, rank, dist, sim_cls=FakeSim)
        q.put((rank, mode, fallback, S.args))
    except bench.ShardBuildError as e:
        q.put((rank, "error", str(e), None))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_make_sim_two_ranks(fail_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if fail_rank is None:
        for rank, mode, fallback, a in res:
            assert mode == "sharded2-rccl" and fallback is None
            assert a == (64, 10, 1, 2, rank, b"\x07" * 128)  # one shard each, rank 0's id
    else:
        for rank, mode, err, a in res:
            assert mode == "error" and "rank 1: no device" in err  # every rank, not only rank 1
            assert a is None


class FakeFailSim:
    """Stands in for a shard of a config-5 run: the cluster-wide convergence
    flag is up from round 3, but this rank's view shows every failed node
    faulty only from round `done_round[rank]`."""
    done_round = {0: 3, 1: 6}

    def __init__(self, n, seed, churn_k=None, shards=1, rank=None, unique_id=None, failures=None, storm=None, arena_entries=0):
        import numpy as np
        self.n, self.rank, self.r = n, rank, 0
        self.dead = failures[0]
        self.np = np

    @staticmethod
    def unique_id():
        return b"\x01" * 128

    def shard_range(self):
        h = self.n // 2
        return (0, h) if self.rank == 0 else (h, self.n)

    def sync(self):
        pass

    def enable_timing(self, on, stages=None):
        pass

    def counters(self):
        return {"evaluated": 10 * self.r, "applied": self.r, "full_syncs": 0, "messages": 2 * self.r}

    def round(self, churn=True):
        self.r += 1
        return {"evaluated": 10, "applied": 1, "full_syncs": 0, "waves": 6, "converged": int(self.r >= 3)}

    def view(self, v):
        st = self.np.ones(self.n, dtype=self.np.uint8)
        if self.r >= self.done_round[self.rank]:
            st[self.dead] = 3
        return st, self.np.zeros(self.n, dtype=self.np.uint64)

    def view_counts(self):
        vc = self.np.zeros((self.n, 6), dtype=self.np.uint32)
        nf = len(self.dead) if self.r >= self.done_round[self.rank] else 0
        vc[:, 1] = self.n - nf
        vc[:, 3] = nf
        vc[:, 5] = self.n - len(self.dead)
        return vc

    def kernel_times(self):
        return {"merge_ping": (1.0, 1)}

    def info(self, v):
        return {"ring_servers": self.n - len(self.dead)}

    def checksums(self):
        return self.np.zeros(self.n, dtype=self.np.uint32)

    def exchange_stats(self):
        return {"ms": 0.0, "bytes_sent": 0, "rounds": self.r}

    def close(self):
        pass


def _fail_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import io
    import contextlib
    import json
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = types.SimpleNamespace(seed=3, shards=1, nodes=64, churn=None, fail_frac=0.1, max_rounds=50,
                                 storm_ppm=1000, storm_rounds=2)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = bench.run_failure(args, world, rank, dist, sim_cls=FakeFailSim)
    dist.destroy_process_group()
    q.put((rank, json.loads(json.dumps(out)) if rank == 0 else None))


def test_failure_workload_two_ranks_agree_on_convergence():
    """bench.py --workload failure on 2 ranks: the stop decision is the AND over
    ranks (no rank leaves the round loop while another still runs rounds), and
    rank 0 reports the round at which both saw every failed node faulty."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    out = res[0]
    assert out["value"] == 6 and out["steps"] == 6 and out["first_agreement_round"] == 3
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "sharded2-rccl"
    assert out["end_state"]["every_failed_faulty"] and out["end_state"]["every_ring_holds_live_servers"]
