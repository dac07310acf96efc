"""Where the merges' log-position checks go (a -DRP_DIAG_APPLY build, e.g.
tools/build_variant.sh diagapply -DRP_DIAG_APPLY, loaded via RINGPOP_HIP_LIB):
per applied change of config 4 in steady state, whether its view cell named a
log position, whether that position was inside the window (a log-slot read),
and what the slot held (tombstone / live makeAlive entry -> origin-table read /
the address's own live entry -> overwritten in place).
usage: python tools/apply_diag.py [nodes] [rounds] [measured]"""
import json
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ringpop_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
pre = int(sys.argv[2]) if len(sys.argv) > 2 else 60
meas = int(sys.argv[3]) if len(sys.argv) > 3 else 10
S = ringpop_amd.Sim(n, 2024, churn_k=-(-n // 100))
S.run(pre)
S.sync()
c0 = S.counters()
S.run(meas)
S.sync()
c1 = S.counters()
d = {k: c1[k] - c0[k] for k in c1}
names = ["applied", "cell_names_a_position", "position_in_window_slot_read", "slot_tombstone",
         "slot_live_makealive_origin_read", "overwritten_in_place"]
out = {nm: d[f"diag{i}"] / meas for i, nm in enumerate(names)}
out["applied_counter_per_round"] = d["applied"] / meas
print(json.dumps(out))
