"""The RCCL leg of sharded simulations: G processes, one GPU
and one shard each (rp_sim_create_rank: ncclAllGather, grouped
ncclSend/ncclRecv all-to-alls, ncclAllReduce, ncclBroadcast), must equal the
in-process G-shard run -- per-round counters, every node's checksum, and
sampled nodes' views, member orders and dissemination tables -- for config 4
at 4,096 nodes and for a fault run (fail-stops + a partition: ping-req waves,
escapes with their origin records and full syncs cross the ranks).

Needs >= G visible GPUs: skipped on a one-GPU box (RCCL refuses two ranks on
one device), run by the driver on an 8-GPU node.
"""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import rccl_ranks  # noqa: E402


def _visible_gpus():
    try:
        import torch
        return torch.cuda.device_count()  # (does not initialise the GPU on this image)
    except Exception:  # noqa: BLE001
        return 0


@pytest.mark.timeout(900)
@pytest.mark.parametrize("G,n,rounds,faults", [(2, 4096, 12, False), (2, 4096, 16, True),
                                               (4, 4096, 12, False), (8, 4096, 16, True)])
def test_rccl_ranks_match_in_process_shards(G, n, rounds, faults):
    if _visible_gpus() < G:
        pytest.skip(f"needs {G} visible GPUs (RCCL: one rank per device)")
    procs = rccl_ranks.spawn(G, n, rounds, faults)
    try:
        per, cs, views = rccl_ranks.reference(G, n, rounds, faults)
    except BaseException:
        for p in procs:
            p.kill()
        raise
    results = rccl_ranks.collect(procs, timeout=600)
    bad = rccl_ranks.compare(results, per, cs, views, n, faults)
    for d, _ in results:
        if d:
            print(f"rank {d['rank']}: exchange {d['exchange']}")
    assert not bad, "\n".join(bad)
