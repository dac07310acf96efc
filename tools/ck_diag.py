"""Where k_checksums_pc spends its time (a -DRP_DIAG build, e.g.
tools/build_variant.sh diagck -DRP_DIAG -DRP_DIAG_PHASE=9 -- no issue
sections -- loaded via RINGPOP_HIP_LIB): config 4 after a pre-roll, one read
of every node's checksum through the lane path; per role (render wave, hash
wave), shader clocks of work and of waiting at the phase barriers per member.
(The single-wave k_checksums_lanes it also measured was removed in round 5.)
usage: python tools/ck_diag.py [nodes] [preroll]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ringpop_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
pre = int(sys.argv[2]) if len(sys.argv) > 2 else 30
S = ringpop_amd.Sim(n, 2024, churn_k=-(-n // 100))  # (the full read takes the lane path, the rounds' short lists the wave path)
S.run(pre)
S.round(churn=True)
S.sync()
c0 = S.counters()
S.checksums()
S.round(churn=True)  # (block counters are summed at a round's end)
S.sync()
c1 = S.counters()
d = {k: c1[k] - c0[k] for k in c1}
if True:  # k_checksums_pc: every wave, per role, work and barrier-wait clocks per member
    m = max(d["diag4"], 1)
    out = {"nodes": n, "views_hashed": d["checksum_views"], "member_walks": d["diag4"],
           "render": {"work_per_member": d["diag0"] / m, "wait_per_member": d["diag1"] / m},
           "hash": {"work_per_member": d["diag2"] / m, "wait_per_member": d["diag3"] / m},
           "shared_phases": d["diag5"], "phases": m // 4}
print(json.dumps(out))
