"""Static checks of the device-state plumbing (CPU): every pointer field of
SimDev (rp_sim.h) is assigned in the shard setup (rp_sim.hip), so a field
added to the struct and never allocated cannot reach a kernel as a null
pointer; and the host-side check_simdev list names only real fields."""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "ringpop_amd", "csrc")


def _simdev_pointer_fields():
    h = open(os.path.join(CSRC, "rp_sim.h")).read()
    body = h[h.index("struct SimDev {"):h.index("enum {", h.index("struct SimDev {"))]
    fields = []
    for line in body.split("\n"):
        line = line.split("//")[0]
        m = re.match(r"\s*(const\s+)?(unsigned\s+long\s+long|[\w:]+)\s*\*\s*([\w, \*]+);", line)
        if m:
            fields += [f.strip().lstrip("*").strip() for f in m.group(3).split(",") if f.strip()]
    return fields


def test_every_simdev_pointer_is_assigned():
    src = open(os.path.join(CSRC, "rp_sim.hip")).read()
    fields = _simdev_pointer_fields()
    assert len(fields) > 90
    missing = [f for f in fields if not re.search(r"\bd\.%s\s*=" % f, src)]
    assert not missing, f"SimDev fields never assigned in setup: {missing}"


def test_check_simdev_names_real_fields():
    src = open(os.path.join(CSRC, "rp_sim.hip")).read()
    body = src[src.index("static void check_simdev"):src.index("void Shard::setup()")]
    named = re.findall(r'\{"(\w+)", d\.(\w+)\}', body)
    assert named and all(a == b for a, b in named)
    fields = set(_simdev_pointer_fields())
    assert {a for a, _ in named} <= fields
    # the fields the round kernels index unconditionally are all listed
    for f in ("view", "dko", "seen", "arena", "sv_word", "target", "resp", "bstats"):
        assert f in {a for a, _ in named}, f


def test_build_tracks_every_header():
    """build.py rebuilds the library when any header a source includes
    changes: its list is the sources' #include closure, and covers every
    header in csrc/ (rp_whash.h was missing from a hand list)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("rp_build", os.path.join(os.path.dirname(CSRC), "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    listed = {os.path.normpath(h) for h in b.HEADERS}
    for f in os.listdir(CSRC):
        if f.endswith(".h"):
            assert f in listed, f"{f} is not tracked by build.py"
    assert os.path.normpath(os.path.join("..", "..", "include", "ringpop_hip.h")) in listed
