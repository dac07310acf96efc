"""The RCCL transport of the rank path (rp::NcclXport: in-place
ncclAllGather, ncclAllReduce, a grouped ncclSend/ncclRecv with every rank,
ncclBroadcast) through rp_comm_selftest, on buffers whose contents every rank
predicts.  One rank runs on the one-GPU box (sends and receives to itself), so
the library's RCCL calls execute on every GPU test run; with G >= 2 visible
GPUs the same check runs in G processes (one per GPU, spawned before this
process touches the device)."""
import ctypes
import os
import subprocess
import sys
import tempfile
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _selftest(nranks, rank, uid, words):
    from ringpop_amd._lib import check, lib
    bad = ctypes.c_uint32(0xFFFFFFFF)
    buf = ctypes.create_string_buffer(bytes(uid), 128)
    check(lib().rp_comm_selftest(nranks, rank, buf, words, ctypes.byref(bad)))
    return bad.value


@pytest.mark.timeout(120)
@pytest.mark.parametrize("words", [1, 1000, 1 << 20])
def test_rccl_transport_one_rank(gpu_lib, words):
    import ringpop_amd
    from ringpop_amd._lib import check, lib
    check(lib().rp_set_device(0))
    assert _selftest(1, 0, ringpop_amd.Sim.unique_id(), words) == 0


CHILD = r"""
import os, sys, time
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
rank, G, idfile = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
from ringpop_amd._lib import check, lib
import ringpop_amd
check(lib().rp_set_device(rank))
if rank == 0:
    uid = ringpop_amd.Sim.unique_id()
    open(idfile + ".tmp", "wb").write(uid)
    os.rename(idfile + ".tmp", idfile)
else:
    t0 = time.time()
    while not os.path.exists(idfile):
        if time.time() - t0 > 60:
            raise SystemExit("no id")
        time.sleep(0.05)
    uid = open(idfile, "rb").read()
import test_gpu_rccl_selftest as t
print("bad", t._selftest(G, rank, uid, 4097), flush=True)
"""


@pytest.mark.timeout(300)
@pytest.mark.parametrize("G", [2, 8])
def test_rccl_transport_g_ranks(G):
    import torch
    if torch.cuda.device_count() < G:
        pytest.skip(f"needs {G} visible GPUs (RCCL: one rank per device)")
    d = tempfile.mkdtemp()
    idfile = os.path.join(d, "uid")
    code = CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r), str(G), idfile], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(G)]
    outs = []
    t0 = time.time()
    for p in procs:
        try:
            o, e = p.communicate(timeout=max(10, 240 - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, e[-2000:]
        assert o.strip().splitlines()[-1] == "bad 0"
