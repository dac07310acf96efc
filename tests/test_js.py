"""The JavaScript host (js/): N-API addon over the C ABI + drop-in classes."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def build_addon():
    from ringpop_amd import build
    build.build()
    js = os.path.join(ROOT, "js")
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-I/usr/include/node", "-o",
                    os.path.join(js, "ringpop_hip.node"), os.path.join(js, "ringpop_napi.c"),
                    "-L" + os.path.join(ROOT, "ringpop_amd"), "-lringpop_hip",
                    "-Wl,-rpath,$ORIGIN/../ringpop_amd"], check=True)


def run_node(script):
    return subprocess.run([NODE, script], capture_output=True, text=True, timeout=600, cwd=ROOT)


def test_addon_loads_and_fails_loudly_without_gpu():
    build_addon()
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    r = subprocess.run([NODE, "-e", "var r=require('./js/index.js');"
                        "var names=['hash32','hash32Batch','ringCreate','ringAddRemove','ringLookup','ringLookupN','ringGroup',"
                        "'simCreate','simRound','simRunAsync','simLoadAddresses','simSetViews','simJoin','simChecksums','simView','simChanges','simPingBody','simHandlePing',"
                        "'simUpdate','nodeCreate','memberUpdate','memberSet','memberSetOrder','dissRecord','dissIssue',"
                        "'dissIssueReceiver','dissFullSync','dissChanges'];"
                        "names.forEach(function(n){ if (typeof r.addon[n] !== 'function') throw new Error(n); });"
                        "try { r.farmhash.hash32('x'); process.exit(3); } catch (e) { process.exit(e.code === '-2' ? 0 : 4); }"],
                       capture_output=True, text=True, cwd=ROOT)
    if r.returncode == 3:
        pytest.skip("a GPU is present: the hash ran")
    assert r.returncode == 0, r.stdout + r.stderr


def test_addon_rejects_malformed_typed_arrays():
    """Argument validation in the N-API layer, before any library call (no GPU
    needed).  profiles/pytest_gpu_r02a.txt records node dying with SIGSEGV in
    tests/js/test_hashring.js while the addon's `opt_u32` still returned NULL
    together with the length of a typed array of the wrong element type, and
    ringAddRemove passed custom replica-hash arrays on without checking their
    length (both fixed in fd9631b): a NULL pointer or a short array travelled
    with a length into the library.  Each call below must throw a TypeError /
    RangeError from the addon, never reach the device, never crash."""
    build_addon()
    script = r"""
var r = require('./js/index.js'), a = r.addon, bad = 0;
function expect(kind, f, what) {
    try { f(); } catch (e) { if (e instanceof kind) return; console.log(what, 'threw', e.name, e.message); bad++; return; }
    console.log(what, 'did not throw'); bad++;
}
expect(TypeError, function () { a.ringLookupHashes(null, new Int32Array(4)); }, 'lookupHashes(Int32Array)');
expect(TypeError, function () { a.ringLookupHashes(null, new Float64Array(4)); }, 'lookupHashes(Float64Array)');
expect(TypeError, function () { a.ringLookupN(null, new Int32Array(2), 3); }, 'lookupN(Int32Array)');
expect(TypeError, function () { a.ringGroup(null, new Uint8Array(9)); }, 'group(Uint8Array)');
expect(RangeError, function () { a.ringAddRemove(null, ['x', 'y'], [], new Uint32Array(150), undefined, 100); },
       'addRemove(short add hashes)');
expect(RangeError, function () { a.ringAddRemove(null, [], ['x'], undefined, new Uint32Array(101), 100); },
       'addRemove(long remove hashes)');
expect(RangeError, function () { a.ringAddRemove(null, ['x'], [], new Int32Array(100), undefined, 100); },
       'addRemove(Int32Array hashes)');
expect(TypeError, function () { a.memberSetOrder(null, new Int32Array(3)); }, 'memberSetOrder(Int32Array)');
expect(TypeError, function () { a.memberSetOrder(null, [0, 1, 2]); }, 'memberSetOrder(Array)');
process.exit(bad ? 1 : 0);
"""
    r = subprocess.run([NODE, "-e", script], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_js_hashring_parity():
    build_addon()
    r = run_node(os.path.join(ROOT, "tests", "js", "test_hashring.js"))
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_js_sim_parity():
    build_addon()
    r = run_node(os.path.join(ROOT, "tests", "js", "test_sim.js"))
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_js_membership_dissemination_parity():
    """The JS drop-in Membership / Dissemination / HashRing of one instance
    against the reference's operation sequences, config 1 and rules table."""
    build_addon()
    r = run_node(os.path.join(ROOT, "tests", "js", "test_node.js"))
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_js_wire_bridge():
    build_addon()
    r = run_node(os.path.join(ROOT, "tests", "js", "test_wire.js"))
    assert r.returncode == 0, r.stdout + r.stderr
