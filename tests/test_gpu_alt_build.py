"""The parity suite's core on the library built with every path-selecting
tuning constant off its default (ringpop_amd/build.py VARIANTS["alt"],
libringpop_hip_alt.so): pass-1 and respond unrolls of 4, a 64-entry issue
stash (most written entries gathered from the log in pass 2), two keys per
merge thread, one ping rank before k_phase2, the per-lane checksum render,
no checksum side stream, cross-shard seen masks per 2 nodes, compaction at
2x + 1,024, the ring's 32-bit directory only and every ring update through
the bulk path.  None of them changes a result, so the reference fixtures,
the oracle comparisons and the ring's per-call checks must hold as they do
for the defaults (only the defaults were under the oracle).
The library is loaded in a child pytest (RINGPOP_HIP_LIB), one process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_alt_constants_parity():
    from ringpop_amd import build
    lib = build.build(variant="alt")  # (built by __graft_entry__.build(); up to date here)
    env = dict(os.environ, RINGPOP_HIP_LIB=lib)
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
           "--timeout", "240", "--timeout-method", "thread",
           "tests/test_gpu_parity.py", "tests/test_gpu_ring_incremental.py",
           "-k", "sim_small or storm or lane_per_view or n256 or medium or ring or farmhash"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    tail = (r.stdout[-4000:] + "\n" + r.stderr[-2000:])
    assert r.returncode == 0, tail
    import re
    m = re.search(r"(\d+) passed", r.stdout)
    assert m and int(m.group(1)) >= 30 and "failed" not in r.stdout, tail  # (the selection ran: ~50 tests)
