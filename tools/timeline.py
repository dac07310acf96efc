"""Where a run's wall time goes, from rocprofv3 --kernel-trace (and optional
--memory-copy-trace) CSVs: busy time (union of kernel and copy intervals) vs
idle gaps, the largest gaps with the kernels around them, and per-kernel
totals over the window.  Experiments only.

usage: timeline.py <kernel_trace.csv> [memory_copy_trace.csv] [--skip FRAC]
  --skip FRAC: ignore the first FRAC of the run (setup), default 0.3
"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
skip = 0.3
if "--skip" in sys.argv:
    skip = float(sys.argv[sys.argv.index("--skip") + 1])
    args = [a for a in args if a != str(skip)]
ev = []
for r in csv.DictReader(open(args[0])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("rp::", "")))
if len(args) > 1:
    for r in csv.DictReader(open(args[1])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", r.get("Kind", "?"))))
ev.sort()
t0, t1 = ev[0][0], max(e[1] for e in ev)
lo = t0 + int((t1 - t0) * skip)
ev = [e for e in ev if e[0] >= lo]
busy, cur_s, cur_e = 0, None, None
gaps = []
prev_name = None
for s, e, k in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, k))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = k
busy += cur_e - cur_s
wall = cur_e - ev[0][0]
print(f"window {wall / 1e6:.2f} ms: busy {busy / 1e6:.2f} ms ({100 * busy / wall:.1f} %), idle {(wall - busy) / 1e6:.2f} ms in {len(gaps)} gaps")
big = sorted(gaps, reverse=True)[:15]
print("largest gaps (us, before -> after):")
for g, a, b in big:
    print(f"  {g / 1e3:9.1f}  {a} -> {b}")
hist = defaultdict(int)
for g, _, _ in gaps:
    hist[min(6, max(0, len(str(int(g / 1e3)))))] += g
print("idle by gap size: " + ", ".join(f"<{10 ** k}us {v / 1e6:.2f} ms" for k, v in sorted(hist.items())))
tot = defaultdict(lambda: [0, 0])
for s, e, k in ev:
    tot[k][0] += e - s
    tot[k][1] += 1
print(f"{'kernel/copy':40s} {'calls':>7s} {'total_ms':>9s}")
for k, (t, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:30]:
    print(f"{k[:40]:40s} {c:7d} {t / 1e6:9.2f}")
