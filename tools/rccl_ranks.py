"""Multi-process check of the RCCL exchange path (rp_sim_create_rank): G
processes, one shard each, against the in-process G-shard run.  On a box with
fewer GPUs than ranks the processes share device 0 (RCCL may refuse that).

usage: python tools/rccl_ranks.py [G] [n] [rounds]
RP_FAULTS=1: every 10th node fail-stops at round 0 and a partition splits the
cluster for rounds 3-12 (ping-req waves and full syncs cross the ranks)."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def faults(n):
    if os.environ.get("RP_FAULTS") != "1":
        return {}
    return {"failures": {0: list(range(0, n, 10))}, "partition": {"start": 3, "end": 12, "split": n // 3}}


def child(G, n, rounds, rank, idfile, ndev):
    import ringpop_amd
    from ringpop_amd._lib import check, lib
    check(lib().rp_set_device(rank % ndev))
    if rank == 0:
        uid = ringpop_amd.Sim.unique_id()
        with open(idfile + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(idfile + ".tmp", idfile)
    else:
        t0 = time.time()
        while not os.path.exists(idfile):
            if time.time() - t0 > 60:
                raise SystemExit("no unique id")
            time.sleep(0.05)
        uid = open(idfile, "rb").read()
    S = ringpop_amd.Sim(n, 2024, churn_k=-(-n // 100), shards=G, rank=rank, unique_id=uid, **faults(n))
    per = []
    for r in range(rounds):
        st = S.round(churn=True)
        per.append([st["evaluated"], st["applied"], st["full_syncs"], st["messages"], st["converged"]])
    lo, hi = S.shard_range()
    cs = S.checksums()[lo:hi].tolist()
    print(json.dumps({"rank": rank, "per": per, "lo": lo, "cs": cs, "x": S.exchange_stats()}), flush=True)
    S.close()


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    if len(sys.argv) > 4:
        return child(G, n, rounds, int(sys.argv[4]), sys.argv[5], int(sys.argv[6]))
    ndev = int(os.environ.get("RP_NDEV", "1"))
    idfile = os.path.join(tempfile.mkdtemp(), "uid")
    # the ranks start before this process touches the GPU
    procs = [subprocess.Popen([sys.executable, __file__, str(G), str(n), str(rounds), str(r), idfile, str(ndev)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(G)]
    import ringpop_amd
    ref = ringpop_amd.Sim(n, 2024, churn_k=-(-n // 100), shards=G, **faults(n))
    rper = []
    for r in range(rounds):
        st = ref.round(churn=True)
        rper.append([st["evaluated"], st["applied"], st["full_syncs"], st["messages"], st["converged"]])
    rcs = ref.checksums().tolist()
    ref.close()
    ok = True
    for p in procs:
        out, err = p.communicate(timeout=300)
        if p.returncode != 0:
            print("rank failed:", p.returncode, err[-2000:])
            ok = False
            continue
        d = json.loads(out.strip().splitlines()[-1])
        dead = set(faults(n).get("failures", {}).get(0, []))
        keep = [i for i in range(len(d["cs"])) if d["lo"] + i not in dead]
        same = d["per"] == rper and [d["cs"][i] for i in keep] == [rcs[d["lo"] + i] for i in keep]
        print(f"rank {d['rank']}: matches in-process shards: {same}; exchange {d['x']}")
        ok &= same
    print("RCCL ranks OK" if ok else "RCCL ranks MISMATCH/FAILED")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
