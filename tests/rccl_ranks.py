"""Multi-process check of the RCCL exchange path (rp_sim_create_rank): G
processes, one shard and one GPU each, against the in-process G-shard run
(rp_sim_create_shards, exchanges as device copies; itself bit-identical to
one shard).  Used by tests/test_gpu_rccl.py; runnable by hand:

    python tests/rccl_ranks.py G n rounds [faults]

faults = 1: every 10th node fail-stops at round 0 and a partition splits the
cluster for rounds 3-12, so ping-req waves, their escapes (suspect/faulty
origins) and full syncs cross the ranks.

The ranks are fresh child processes started before this process touches the
GPU (and never exec'd from a GPU process); rank 0 writes the RCCL unique id to
a file the others poll.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def sim_kwargs(n, faults):
    kw = {"churn_k": -(-n // 100)}
    if faults:
        kw["failures"] = {0: list(range(0, n, 10))}
        kw["partition"] = {"start": 3, "end": 12, "split": n // 3}
    return kw


def _stats(st):
    return [st[k] for k in ("evaluated", "applied", "full_syncs", "messages", "waves", "converged")]


def child(G, n, rounds, faults, rank, idfile):
    import ringpop_amd
    from ringpop_amd._lib import check, lib
    check(lib().rp_set_device(rank))
    if rank == 0:
        uid = ringpop_amd.Sim.unique_id()
        with open(idfile + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(idfile + ".tmp", idfile)
    else:
        t0 = time.time()
        while not os.path.exists(idfile):
            if time.time() - t0 > 120:
                raise SystemExit("rank %d: no unique id after 120 s" % rank)
            time.sleep(0.05)
        with open(idfile, "rb") as f:
            uid = f.read()
    S = ringpop_amd.Sim(n, 2024, shards=G, rank=rank, unique_id=uid, **sim_kwargs(n, faults))
    S.enable_timing(True)
    per = [_stats(S.round(churn=True)) for _ in range(rounds)]
    lo, hi = S.shard_range()
    cs = S.checksums()[lo:hi].tolist()
    views = {}
    for v in (lo, (lo + hi) // 2, hi - 1):
        st, inc = S.view(v)
        views[v] = [st.tolist(), inc.tolist(), S.members(v).tolist(), S.changes(v).tolist()]
    print(json.dumps({"rank": rank, "per": per, "lo": lo, "hi": hi, "cs": cs, "views": views,
                      "exchange": S.exchange_stats()}), flush=True)
    S.close()


def run_loop(G, n, rounds, faults):
    """The same G ranks as threads of this process on the current device
    (rp_sim_create_rank_loop: the rank code with device-copy collectives);
    results in collect()'s format."""
    import threading

    import ringpop_amd
    from ringpop_amd.sim import Loop
    loop = Loop(G)
    sims = [ringpop_amd.Sim(n, 2024, shards=G, rank=r, loop=loop, **sim_kwargs(n, faults)) for r in range(G)]
    out = [None] * G

    def rank_main(r):
        S = sims[r]
        try:
            S.enable_timing(True)
            per = [_stats(S.round(churn=True)) for _ in range(rounds)]
            lo, hi = S.shard_range()
            cs = S.checksums()[lo:hi].tolist()
            views = {}
            for v in (lo, (lo + hi) // 2, hi - 1):
                st, inc = S.view(v)
                views[v] = [st.tolist(), inc.tolist(), S.members(v).tolist(), S.changes(v).tolist()]
            out[r] = ({"rank": r, "per": per, "lo": lo, "hi": hi, "cs": cs, "views": views,
                       "exchange": S.exchange_stats()}, "")
        except Exception as e:  # noqa: BLE001 - reported per rank
            out[r] = (None, "rank %d: %r" % (r, e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for S in sims:
        S.close()
    loop.close()
    return out


def spawn(G, n, rounds, faults):
    """Start the G rank processes (call before this process uses the GPU)."""
    idfile = os.path.join(tempfile.mkdtemp(prefix="rccl_uid_"), "uid")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--child", str(G), str(n), str(rounds),
                              "1" if faults else "0", str(r), idfile],
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=ROOT)
            for r in range(G)]


def reference(G, n, rounds, faults):
    """The in-process G-shard run on the current device."""
    import ringpop_amd
    ref = ringpop_amd.Sim(n, 2024, shards=G, **sim_kwargs(n, faults))
    per = [_stats(ref.round(churn=True)) for _ in range(rounds)]
    cs = ref.checksums().tolist()
    views = {}
    for r in range(G):
        lo, hi = r * n // G, (r + 1) * n // G
        for v in (lo, (lo + hi) // 2, hi - 1):
            st, inc = ref.view(v)
            views[v] = [st.tolist(), inc.tolist(), ref.members(v).tolist(), ref.changes(v).tolist()]
    ref.close()
    return per, cs, views


def collect(procs, timeout=600):
    """[(rank result dict | None, error text)] in rank order."""
    out = []
    t_end = time.time() + timeout
    for p in procs:
        try:
            so, se = p.communicate(timeout=max(1.0, t_end - time.time()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        if p.returncode != 0:
            out.append((None, "rank exit %d: %s" % (p.returncode, se[-3000:])))
        else:
            out.append((json.loads(so.strip().splitlines()[-1]), ""))
    return out


def compare(results, per, cs, views, n, faults):
    """Mismatch descriptions (empty: the RCCL ranks equal the in-process shards)."""
    bad = []
    dead = set(sim_kwargs(n, faults).get("failures", {}).get(0, []))
    for d, err in results:
        if d is None:
            bad.append(err)
            continue
        r, lo = d["rank"], d["lo"]
        if d["per"] != per:
            k = next(i for i, (a, b) in enumerate(zip(d["per"], per)) if a != b)
            bad.append("rank %d: round %d counters %s != %s" % (r, k, d["per"][k], per[k]))
        keep = [i for i in range(len(d["cs"])) if lo + i not in dead]
        if [d["cs"][i] for i in keep] != [cs[lo + i] for i in keep]:
            bad.append("rank %d: checksums differ" % r)
        for v, got in d["views"].items():
            if int(v) not in dead and got != views[int(v)]:
                bad.append("rank %d: node %s view/members/changes differ" % (r, v))
    return bad


def main():
    G, n, rounds = (int(x) for x in sys.argv[1:4])
    faults = len(sys.argv) > 4 and sys.argv[4] == "1"
    procs = spawn(G, n, rounds, faults)
    per, cs, views = reference(G, n, rounds, faults)
    results = collect(procs)
    bad = compare(results, per, cs, views, n, faults)
    for d, _ in results:
        if d:
            print("rank %d: exchange %s" % (d["rank"], d["exchange"]))
    print("\n".join(bad) if bad else "RCCL ranks == in-process shards")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1", int(sys.argv[6]), sys.argv[7])
    else:
        main()
