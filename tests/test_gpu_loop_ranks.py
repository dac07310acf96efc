"""The rank path of sharded simulations on one GPU: G ranks of
rp_sim_create_rank's code -- one shard each, driven from their own host
threads -- exchange through the loopback transport (rp_sim_create_rank_loop:
the collectives as device copies after a rendezvous of the rank threads), and
must equal the in-process G-shard run: per-round counters, every node's
checksum, and sampled nodes' views, member orders and dissemination tables,
for config 4 at 4,096 nodes and a fault run (fail-stops + a partition:
ping-req waves, escapes, settled masks, full syncs).  Only the transport
differs from the RCCL ranks of tests/test_gpu_rccl.py."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import rccl_ranks  # noqa: E402


@pytest.fixture(scope="module")
def rp(gpu_lib):
    import ringpop_amd
    return ringpop_amd


@pytest.mark.timeout(600)
@pytest.mark.parametrize("G,n,rounds,faults", [(2, 4096, 12, False), (2, 4096, 16, True),
                                               (4, 4096, 12, False), (8, 4096, 16, True)])
def test_loop_ranks_match_in_process_shards(rp, G, n, rounds, faults):
    results = rccl_ranks.run_loop(G, n, rounds, faults)
    per, cs, views = rccl_ranks.reference(G, n, rounds, faults)
    bad = rccl_ranks.compare(results, per, cs, views, n, faults)
    assert not bad, "\n".join(bad)
    sent = [d["exchange"]["bytes_sent"] for d, _ in results]
    assert all(b > 0 for b in sent), sent  # (every rank exchanged over the transport)
