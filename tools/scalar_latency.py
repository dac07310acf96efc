"""Per-call latency of the drop-in's scalar entry points against the batched
ones: HashRing.lookup one key per call vs lookup_batch,
farmhash hash32 of a short key and of a config-1-sized checksum string.
Prints one JSON object.  GPU box only."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ringpop_amd as rp


def per_call(fn, reps):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps


def main():
    ring = rp.HashRing()
    servers = [f"10.{i // 250}.{i % 250}.1:3000" for i in range(1000)]
    ring.addRemoveServers(servers, None)
    rng = np.random.default_rng(1)
    keys = [str(x) for x in rng.integers(0, 10**12, size=1_000_000)]
    out = {}
    it = iter(keys * 2)
    out["lookup_scalar_us"] = per_call(lambda: ring.lookup(next(it)), 2000) * 1e6
    t = time.perf_counter()
    ring.lookup_batch(keys)
    out["lookup_batch_1M_ns_per_key"] = (time.perf_counter() - t) / len(keys) * 1e9
    out["hash32_short_us"] = per_call(lambda: rp.hash32("10.0.0.1:3000alive1434401518824"), 2000) * 1e6
    big = ";".join(f"10.{i // 250}.{i % 250}.1:3000alive1434401518824" for i in range(65536))
    out["hash32_string_bytes"] = len(big)
    out["hash32_string_ms"] = per_call(lambda: rp.hash32(big), 20) * 1e3
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
