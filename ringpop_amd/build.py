"""Build libringpop_hip.so (gfx950) in-tree with hipcc.

No cmake: one hipcc compile per .hip source (in parallel), one link.
"""
import json
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libringpop_hip.so")
SOURCES = ["rp_capi.hip", "rp_ring.hip", "rp_sim.hip", "rp_node.hip", "rp_calib.hip"]
_INCLUDE_RE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def included_headers(sources=SOURCES, csrc=CSRC):
    """Every quoted header the sources include, transitively (paths relative
    to csrc), so an edit to any of them rebuilds the library."""
    seen, todo = set(), [os.path.join(csrc, s) for s in sources]
    while todo:
        path = todo.pop()
        with open(path) as f:
            text = f.read()
        for inc in _INCLUDE_RE.findall(text):
            h = os.path.normpath(os.path.join(os.path.dirname(path), inc))
            if h not in seen and os.path.exists(h):
                seen.add(h)
                todo.append(h)
    return sorted(os.path.relpath(h, csrc) for h in seen)


HEADERS = included_headers()
ARCH = os.environ.get("RINGPOP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall", "-Wno-unused-function"]
# Builds of the same sources with other compile-time settings, each its own
# library next to the product (loaded through RINGPOP_HIP_LIB):
#  diag -- in-kernel cycle stamps (RP_DIAG);
#  alt  -- every tuning constant that selects a code path set off its default
#          (unrolls, stash size, keys per thread, ping-rank split, checksum
#          render and side stream, compaction thresholds, seen-mask groups,
#          the ring's 16-bit directory and incremental path), so that the
#          parity suite runs the non-default paths too
#          (tests/test_gpu_alt_build.py).  None of them changes a result.
VARIANTS = {
    "diag": ["-DRP_DIAG"],
    "alt": ["-DRP_ISSUE_UNR_P1=4", "-DRP_ISSUE_UNR=4", "-DRP_ISSUE_STASH=64", "-DRP_ISSUE_P2U=1", "-DRP_SETTLED_PF=0",
            "-DRP_KPT=2", "-DRP_P2_SPLIT=1", "-DRP_CKP_SHARED=0", "-DRP_CK_SIDE=0", "-DRP_SEEN_GROUP_LOG=1",
            "-DRP_COMPACT_MUL=2u", "-DRP_COMPACT_ADD=1024u", "-DRP_LOOKUP_DIR16=0", "-DRP_RING_INCR_MAX_POINTS=0"],
}


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def _stamp(flags):
    """What the objects depend on besides the sources: compiler, arch, flags."""
    return json.dumps({"hipcc": os.path.realpath(HIPCC), "arch": ARCH, "flags": flags,
                       "sources": SOURCES}, sort_keys=True)


def variant_lib(variant):
    return LIB.replace(".so", "_" + variant + ".so")


def build(force=False, verbose=False, diag=False, variant=None):
    """variant (or diag=True for "diag"): one of VARIANTS -> libringpop_hip_<variant>.so."""
    variant = "diag" if diag else variant
    obj_dir, lib = (OBJ + "_" + variant, variant_lib(variant)) if variant else (OBJ, LIB)
    flags = FLAGS + (VARIANTS[variant] if variant else [])
    os.makedirs(obj_dir, exist_ok=True)
    stamp_path = lib + ".stamp"
    stamp = _stamp(flags)
    old = open(stamp_path).read() if os.path.exists(stamp_path) else None
    if old is not None and old != stamp:
        force = True  # another compiler, arch or flag set: rebuild everything
    hdr_time = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    src_time = max([hdr_time] + [_mtime(os.path.join(CSRC, s)) for s in SOURCES])
    if not force and old == stamp and _mtime(lib) >= src_time:
        return lib  # up to date (objects do not travel to the GPU box; the library does)
    objs, jobs = [], []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(obj_dir, src.replace(".hip", ".o"))
        objs.append(o)
        if force or _mtime(o) < max(_mtime(s), hdr_time):
            jobs.append([HIPCC, *flags, "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
        return r

    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "8"))))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(run, jobs))
    if jobs or force or _mtime(lib) < max(_mtime(o) for o in objs):
        run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", lib, *objs, "-L/opt/rocm/lib", "-lrccl",
             "-Wl,-rpath,/opt/rocm/lib"])
    with open(stamp_path, "w") as f:
        f.write(stamp)
    return lib


if __name__ == "__main__":
    v = next((a[2:] for a in sys.argv[1:] if a[2:] in VARIANTS), None)  # --diag / --alt
    print(build(force="--force" in sys.argv, verbose=True, variant=v))
