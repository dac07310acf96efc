"""Per-round issue/exchange volumes at full size: single shard vs G in-process
shards (written = entries that pass the seen filter and are stored/shipped)."""
import json
import math
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ringpop_amd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
G = int(sys.argv[2]) if len(sys.argv) > 2 else 2
W, K = 20, 5
k = math.ceil(0.01 * n)
for shards in (1, G):
    S = ringpop_amd.Sim(n, 2024, churn_k=k, shards=shards)
    S.run(W)
    S.sync()
    c0 = S.counters()
    S.enable_timing(True)
    S.run(K)
    S.sync()
    c1 = S.counters()
    d = {key: (c1[key] - c0[key]) / K for key in c1}
    x = S.exchange_stats()
    print(json.dumps({"shards": shards, "per_round": {key: d[key] for key in (
        "evaluated", "eval_ping_merge", "eval_resp_merge", "emitted_send_issue", "written_send_issue",
        "emitted_recv_issue", "written_recv_issue", "scanned_send_issue", "scanned_recv_issue")},
        "exchange_bytes_per_round": x["bytes_sent"] / K, "exchange_ms_per_round": x["ms"] / K}), flush=True)
    S.close()
