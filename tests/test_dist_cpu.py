"""World-size-2 gloo tests (CPU) of bench.py's multi-GPU host logic: the RCCL
communicator id is broadcast from rank 0, every rank builds its shard, and if
any rank cannot, all ranks fall back to replicas together (no rank is left
waiting in a collective)."""
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

    def __init__(self, n, seed, churn_k=None, shards=1, rank=None, unique_id=None):
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
    S, mode, fallback = bench.make_sim(args, 64, 1, world, rank, rank, dist, sim_cls=FakeSim)
    q.put((rank, mode, fallback, S.args))
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
        for rank, mode, fallback, a in res:
            assert mode == "replicas" and "rank 1: no device" in fallback
            assert a == (64, 10 + rank, 1, 1, None, None)  # independent replica per rank
