"""Device-resident simulation of N ringpop instances (rp_sim_* C ABI)."""
import ctypes

import numpy as np

from ._lib import RoundStats, SimConfig, check, lib, ptr

KERNEL_CATEGORIES = ("churn", "issue", "merge_ping", "merge_resp", "checksum", "other")
STATUS_NAMES = {0: None, 1: "alive", 2: "suspect", 3: "faulty", 4: "leave"}


class Loop:
    """rp_loop: the ranks of a `nranks`-rank cluster as threads of this process
    on one GPU (rp_sim_create_rank_loop; the rank code of an RCCL cluster with
    device-copy collectives).  Each rank's Sim is driven from its own thread."""

    def __init__(self, nranks):
        self._h = ctypes.c_void_p()
        self.nranks = nranks
        check(lib().rp_loop_create(nranks, ctypes.byref(self._h)))

    def close(self):
        if self._h:
            lib().rp_loop_destroy(self._h)
            self._h = ctypes.c_void_p()


class Sim:
    def __init__(self, n, seed, churn_k=None, arena_entries=0, snapshot_slots=0, origin_slots=0, failures=None,
                 partition=None, seen_window=0, replica_hash_shift=0, shards=1, rank=None, unique_id=None,
                 storm=None, addresses=None, views=None, joins=None, compact=None, loop=None, prefix_min=0, ck_lane_min=0):
        """shards > 1: the nodes are split into `shards` shards.  With rank=None
        all shards run in this process (rp_sim_create_shards); with a rank, this
        process holds that shard of a one-process-per-GPU cluster whose RCCL
        communicator is named by `unique_id` (rp_sim_create_rank), or -- with
        loop=Loop(shards) -- that rank of a cluster of threads of this process
        (rp_sim_create_rank_loop).
        addresses: the cluster's n address strings in sort order
        (rp_sim_load_addresses); views: (status, incarnation) arrays of shape
        (n, n) for the bootstrap (rp_sim_set_views; status 0 = absent);
        joins: [(round, joiner, [seeds...]), ...] (rp_sim_join);
        compact: (mul, add) log-compaction thresholds (testing; None = auto);
        prefix_min: the window shrink that triggers the issue's head packing
        beyond the entries it moves (testing; 0 = auto, 512);
        ck_lane_min: checksum lists this long are hashed one view per lane
        (0 = auto; 1 = always, 0xFFFFFFFF = never)."""
        self.n = n
        self.churn_k = -(-n // 100) if churn_k is None else churn_k
        cfg = SimConfig(n=n, churn_k=self.churn_k, seed=seed, arena_entries=arena_entries,
                        snapshot_slots=snapshot_slots, origin_slots=origin_slots,
                        seen_window=seen_window, replica_hash_shift=replica_hash_shift,
                        compact_mul=compact[0] if compact else 0, compact_add=compact[1] if compact else 0,
                        prefix_min=prefix_min, ck_lane_min=ck_lane_min)
        self._h = ctypes.c_void_p()
        self.shards = shards
        if rank is not None and loop is not None:
            check(lib().rp_sim_create_rank_loop(ctypes.byref(cfg), loop._h, rank, ctypes.byref(self._h)))
        elif rank is not None:
            uid = ctypes.create_string_buffer(bytes(unique_id), 128)
            check(lib().rp_sim_create_rank(ctypes.byref(cfg), shards, rank, uid, ctypes.byref(self._h)))
        elif shards > 1:
            check(lib().rp_sim_create_shards(ctypes.byref(cfg), shards, ctypes.byref(self._h)))
        else:
            check(lib().rp_sim_create(ctypes.byref(cfg), ctypes.byref(self._h)))
        for rnd, ids in (failures or {}).items():
            for v in ids:
                check(lib().rp_sim_fail(self._h, int(v), int(rnd)))
        if partition:
            check(lib().rp_sim_partition(self._h, partition["start"], partition["end"], partition["split"]))
        if storm:  # {"start", "end", "ppm"}: false suspicions (rp_sim_storm)
            check(lib().rp_sim_storm(self._h, storm["start"], storm["end"], storm["ppm"]))
        if addresses is not None:
            self.load_addresses(addresses)
        if joins:
            self.join(joins)
        if views is not None:
            self.set_views(views[0], views[1])

    def join(self, joins):
        """rp_sim_join: [(round, joiner, [seed, ...]), ...] in processing order."""
        k = len(joins)
        sp = max([len(j[2]) for j in joins] + [1])
        ids = np.array([j[1] for j in joins], dtype=np.uint32)
        rounds = np.array([j[0] for j in joins], dtype=np.uint32)
        seeds = np.full((k, sp), -1, dtype=np.int32)
        for i, j in enumerate(joins):
            seeds[i, :len(j[2])] = j[2]
        check(lib().rp_sim_join(self._h, ptr(ids), ptr(rounds), ptr(seeds), k, sp))

    def load_addresses(self, addresses):
        """rp_sim_load_addresses: node i is addresses[i] (sorted, distinct)."""
        bs = [a.encode() if isinstance(a, str) else bytes(a) for a in addresses]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs])
        blob = np.frombuffer(b"".join(bs) or b"\0", dtype=np.uint8)
        check(lib().rp_sim_load_addresses(self._h, ptr(blob), ptr(off), len(bs)))

    def set_views(self, status, incarnation, node_lo=0):
        """rp_sim_set_views for nodes node_lo .. node_lo + len(status): rows of
        member statuses (1..4) and incarnations, shape (count, n)."""
        st = np.ascontiguousarray(status, dtype=np.int32)
        inc = np.ascontiguousarray(incarnation, dtype=np.int64)
        if st.ndim != 2 or st.shape != inc.shape or st.shape[1] != self.n:
            raise ValueError("views: two (count, n) arrays")
        check(lib().rp_sim_set_views(self._h, int(node_lo), st.shape[0], ptr(st), ptr(inc)))

    @staticmethod
    def unique_id():
        """A fresh RCCL communicator id (128 bytes) for rp_sim_create_rank."""
        buf = ctypes.create_string_buffer(128)
        check(lib().rp_comm_unique_id(buf, 128))
        return buf.raw

    def shard_range(self):
        lo, hi = ctypes.c_uint32(0), ctypes.c_uint32(0)
        check(lib().rp_sim_shard_range(self._h, ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    def exchange_stats(self):
        ms, b, r = ctypes.c_double(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(lib().rp_sim_exchange_stats(self._h, ctypes.byref(ms), ctypes.byref(b), ctypes.byref(r)))
        out = {"ms": ms.value, "bytes_sent": b.value, "rounds": r.value}
        if hasattr(lib(), "rp_sim_exchange_shard_bytes"):  # (an older A/B variant may lack it)
            arr, cnt = (ctypes.c_uint64 * 64)(), ctypes.c_int(0)
            check(lib().rp_sim_exchange_shard_bytes(self._h, arr, 64, ctypes.byref(cnt)))
            out["shard_bytes"] = [int(arr[i]) for i in range(min(cnt.value, 64))]
        return out

    def close(self):
        if self._h:
            lib().rp_sim_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def round(self, churn=True):
        st = RoundStats()
        check(lib().rp_sim_round(self._h, 1 if churn else 0, ctypes.byref(st)))
        return st.as_dict()

    def run(self, k, churn=True):
        check(lib().rp_sim_run(self._h, int(k), 1 if churn else 0))

    def sync(self):
        check(lib().rp_sim_sync(self._h))

    def totals(self):
        st = RoundStats()
        check(lib().rp_sim_totals(self._h, ctypes.byref(st)))
        d = st.as_dict()
        d["converged_rounds"] = d.pop("converged")
        return d

    COUNTERS = ("evaluated", "applied", "full_syncs", "messages", "waves", "pings", "eval_ping_merge",
                "applied_ping_merge", "eval_resp_merge", "applied_resp_merge", "scanned_send_issue",
                "emitted_send_issue", "scanned_recv_issue", "emitted_recv_issue", "written_send_issue",
                "written_recv_issue", "touched", "touched_ping_merge", "checksum_views", "compactions_issue",
                "compactions_apply", "prefix_packs", "same_view_issues", "diag0", "diag1", "diag2", "diag3", "diag4", "diag5")

    def counters(self):
        """Cumulative counters: the round statistics, per-kernel unit counts and
        diagnostics (rp_sim_counters); the last entry is converged_rounds."""
        out = np.zeros(64, dtype=np.uint64)
        n = ctypes.c_int(0)
        check(lib().rp_sim_counters(self._h, ptr(out), 64, ctypes.byref(n)))
        d = {k: int(out[i]) for i, k in enumerate(self.COUNTERS[: n.value - 1])}
        d["converged_rounds"] = int(out[n.value - 1])
        return d

    def local_counters(self):
        """counters() of this process's shards only (equal to counters() for one
        shard or all shards in process)."""
        out = np.zeros(64, dtype=np.uint64)
        n = ctypes.c_int(0)
        check(lib().rp_sim_local_counters(self._h, ptr(out), 64, ctypes.byref(n)))
        return {k: int(out[i]) for i, k in enumerate(self.COUNTERS[: n.value - 1])}

    def rounds(self):
        r = ctypes.c_uint32(0)
        check(lib().rp_sim_rounds(self._h, ctypes.byref(r)))
        return r.value

    def checksums(self):
        out = np.zeros(self.n, dtype=np.uint32)
        check(lib().rp_sim_read_checksums(self._h, ptr(out), len(out)))
        return out

    def view_counts(self):
        """Per node: members absent / alive / suspect / faulty / leave and its
        ring server count ([n, 6]; nodes held by other processes are 0)."""
        out = np.zeros((self.n, 6), dtype=np.uint32)
        check(lib().rp_sim_view_counts(self._h, ptr(out), out.size))
        return out

    def view(self, v):
        st = np.zeros(self.n, dtype=np.uint8)
        inc = np.zeros(self.n, dtype=np.uint64)
        check(lib().rp_sim_read_view(self._h, v, ptr(st), ptr(inc), self.n))
        return st, inc

    def members(self, v):
        out = np.zeros(self.n, dtype=np.uint32)
        cnt = ctypes.c_uint32(0)
        check(lib().rp_sim_read_members(self._h, v, ptr(out), len(out), ctypes.byref(cnt)))
        return out[: cnt.value].astype(np.int32)

    def changes(self, v):
        cnt = ctypes.c_uint32(0)
        check(lib().rp_sim_read_changes(self._h, v, None, 0, ctypes.byref(cnt)))
        rows = np.zeros((max(cnt.value, 1), 6), dtype=np.int64)
        check(lib().rp_sim_read_changes(self._h, v, ptr(rows), rows.shape[0], ctypes.byref(cnt)))
        return rows[: cnt.value]

    def info(self, v):
        out = np.zeros(8, dtype=np.int64)
        check(lib().rp_sim_node_info(self._h, v, ptr(out)))
        keys = ("max_pb", "ring_servers", "ring_checksum", "iter_index", "iter_round", "dead", "rng", "timers")
        return dict(zip(keys, out.tolist()))

    def ring_lookup(self, v, hashes):
        h = np.ascontiguousarray(hashes, dtype=np.uint32)
        out = np.zeros(len(h), dtype=np.int32)
        check(lib().rp_sim_ring_lookup(self._h, v, ptr(h), len(h), ptr(out)))
        return out

    def address(self, v):
        buf = ctypes.create_string_buffer(64)
        check(lib().rp_sim_address(self._h, v, buf, 64))
        return buf.value.decode()

    # ---- wire bridge: the node-level ping path between rounds (wire.py codes
    # the JSON); changes are int64 rows (address, status, incarnation,
    # source, source incarnation), -1 / 0 = undefined
    def _rows(self, rows):
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64).reshape(-1, 5))
        return r, len(r)

    def ping_body(self, v):
        """PingSender.send (lib/swim/ping-sender.js:70-76): (changes, checksum, incarnation)."""
        out = np.zeros((self.n, 5), dtype=np.int64)
        cnt, cs, inc = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_uint64(0)
        check(lib().rp_sim_ping_body(self._h, v, ptr(out), self.n, ctypes.byref(cnt), ctypes.byref(cs),
                                     ctypes.byref(inc)))
        return out[: cnt.value], cs.value, inc.value

    def handle_ping(self, v, source, source_inc, checksum, rows):
        """handlePing (server/ping-handler.js:22-40): (response changes, applied, full_sync)."""
        r, k = self._rows(rows)
        out = np.zeros((self.n, 5), dtype=np.int64)
        cnt, ap, fs = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
        check(lib().rp_sim_handle_ping(self._h, v, int(source), int(source_inc), int(checksum) & 0xFFFFFFFF,
                                       ptr(r), k, ptr(out), self.n, ctypes.byref(cnt), ctypes.byref(ap),
                                       ctypes.byref(fs)))
        return out[: cnt.value], ap.value, bool(fs.value)

    def update(self, v, rows):
        """Membership.update at node v (PingSender.onPing, lib/swim/ping-sender.js:36-39): applied count."""
        r, k = self._rows(rows)
        ap = ctypes.c_uint32(0)
        check(lib().rp_sim_update(self._h, v, ptr(r), k, ctypes.byref(ap)))
        return ap.value

    def checksum(self, v):
        """membership.checksum of node v."""
        return int(self.checksums()[v])

    def addresses(self):
        if getattr(self, "_addrs", None) is None:
            self._addrs = [self.address(v) for v in range(self.n)]
        return self._addrs

    def enable_timing(self, on=True, stages=None):
        """Per-stage device time from now on (kernel_times).  stages: the
        KERNEL_CATEGORIES names (and "exchange") to time; None = all.  Each
        timed stage puts two events per launch on the simulation stream."""
        if stages is None:
            check(lib().rp_sim_enable_timing(self._h, 1 if on else 0))
            return
        names = list(KERNEL_CATEGORIES) + ["exchange"]
        mask = 0
        for st in stages:
            mask |= 1 << names.index(st)
        check(lib().rp_sim_enable_timing_stages(self._h, mask if on else 0))

    def kernel_times(self):
        ms = np.zeros(6, dtype=np.float64)
        cnt = np.zeros(6, dtype=np.uint64)
        check(lib().rp_sim_kernel_times(self._h, ptr(ms), ptr(cnt)))
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(KERNEL_CATEGORIES)}

    def side_ms(self):
        """Device ms of the side stream's checksum chains and fullSync decisions
        (beside the ping and response merges; one shard), since enable_timing."""
        ms = np.zeros(1, dtype=np.float64)
        check(lib().rp_sim_side_ms(self._h, ptr(ms)))
        return float(ms[0])
