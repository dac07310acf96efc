"""ctypes binding of include/ringpop_hip.h (libringpop_hip.so).

The library is the product: there is no CPU fallback.  Loading fails loudly
when the shared object is missing, and every entry point raises when the HIP
runtime has no usable GPU.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RINGPOP_HIP_LIB: load another build of the same library (e.g. the RP_DIAG
# diagnostic build, ringpop_amd/build.py --diag)
LIB_PATH = os.environ.get("RINGPOP_HIP_LIB") or os.path.join(_HERE, "libringpop_hip.so")

RP_OK = 0
ERRORS = {-1: "invalid argument", -2: "HIP error", -3: "out of device memory", -4: "unsupported",
          -5: "capacity exceeded", -6: "kernel error"}


class RingpopError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class SimConfig(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("churn_k", ctypes.c_uint32), ("seed", ctypes.c_uint64),
                ("arena_entries", ctypes.c_uint64), ("snapshot_slots", ctypes.c_uint32),
                ("origin_slots", ctypes.c_uint32), ("seen_window", ctypes.c_uint32), ("replica_hash_shift", ctypes.c_uint32),
                ("compact_mul", ctypes.c_uint32), ("compact_add", ctypes.c_uint32), ("prefix_min", ctypes.c_uint32),
                ("ck_lane_min", ctypes.c_uint32)]


class RoundStats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in
                ("evaluated", "applied", "full_syncs", "messages", "waves", "pings", "converged")]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# (name, argtypes) of every entry point declared in include/ringpop_hip.h
_P = ctypes.c_void_p
_U8P = ctypes.POINTER(ctypes.c_uint8)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)
_I32P = ctypes.POINTER(ctypes.c_int32)
_I64P = ctypes.POINTER(ctypes.c_int64)
_SZ = ctypes.c_size_t
SIGNATURES = {
    "rp_last_error": ([], ctypes.c_char_p),
    "rp_abi_version": ([], ctypes.c_int),
    "rp_set_device": ([ctypes.c_int], ctypes.c_int),
    "rp_device_malloc": ([_SZ, ctypes.POINTER(_P)], ctypes.c_int),
    "rp_device_free": ([_P], ctypes.c_int),
    "rp_device_memcpy": ([_P, _P, _SZ, ctypes.c_int], ctypes.c_int),
    "rp_device_synchronize": ([], ctypes.c_int),
    "rp_device_memory": ([ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)], ctypes.c_int),
    "rp_stream_create": ([ctypes.POINTER(_P)], ctypes.c_int),
    "rp_stream_destroy": ([_P], ctypes.c_int),
    "rp_stream_synchronize": ([_P], ctypes.c_int),
    "rp_event_create": ([ctypes.POINTER(_P)], ctypes.c_int),
    "rp_event_record": ([_P, _P], ctypes.c_int),
    "rp_event_elapsed_ms": ([_P, _P, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "rp_event_destroy": ([_P], ctypes.c_int),
    "rp_calibrate": ([_SZ, ctypes.POINTER(ctypes.c_double), ctypes.c_int], ctypes.c_int),
    "rp_device_pci_bus_id": ([ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "rp_hash32": ([_P, _SZ, _U32P], ctypes.c_int),
    "rp_hash32_batch": ([_P, _P, _SZ, _P], ctypes.c_int),
    "rp_hash32_batch_device": ([_P, _P, _SZ, _P, _P], ctypes.c_int),
    "rp_ring_create": ([ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "rp_ring_destroy": ([_P], ctypes.c_int),
    "rp_ring_add_remove": ([_P, _P, _P, _SZ, _P, _P, _P, _SZ, _P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_ring_server_count": ([_P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_ring_has_server": ([_P, _P, _SZ, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_ring_checksum": ([_P, _U32P], ctypes.c_int),
    "rp_ring_server_name": ([_P, ctypes.c_int, ctypes.c_char_p, _SZ, ctypes.POINTER(_SZ)], ctypes.c_int),
    "rp_ring_lookup_batch": ([_P, _P, _P, _SZ, _P], ctypes.c_int),
    "rp_ring_lookup_batch_device": ([_P, _P, _P, _SZ, _P, _P], ctypes.c_int),
    "rp_ring_lookup_hashes": ([_P, _P, _SZ, _P], ctypes.c_int),
    "rp_ring_lookup_n_hashes": ([_P, _P, _SZ, ctypes.c_int, _P, _P], ctypes.c_int),
    "rp_ring_group_keys": ([_P, _P, _P, _SZ, _P, _P, _P, ctypes.POINTER(_SZ)], ctypes.c_int),
    "rp_ring_group_hashes": ([_P, _P, _SZ, _P, _P, _P, ctypes.POINTER(_SZ)], ctypes.c_int),
    "rp_ring_group_device": ([_P, _P, _SZ, _P, _P, _P, ctypes.POINTER(_SZ), _P], ctypes.c_int),
    "rp_ring_points": ([_P, _P, _P, _SZ, ctypes.POINTER(_SZ)], ctypes.c_int),
    "rp_ring_make_keys_device": ([_P, ctypes.c_uint64, _SZ, ctypes.POINTER(_P), ctypes.POINTER(_P), _U64P],
                                 ctypes.c_int),
    "rp_sim_create": ([ctypes.POINTER(SimConfig), ctypes.POINTER(_P)], ctypes.c_int),
    "rp_sim_destroy": ([_P], ctypes.c_int),
    "rp_sim_create_shards": ([ctypes.POINTER(SimConfig), ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "rp_comm_unique_id": ([_P, _SZ], ctypes.c_int),
    "rp_ring_build_ms": ([_P, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
    "rp_ring_profile": ([_P, ctypes.POINTER(ctypes.c_double), ctypes.c_int], ctypes.c_int),
    "rp_comm_selftest": ([ctypes.c_int, ctypes.c_int, _P, ctypes.c_uint32, _U32P], ctypes.c_int),
    "rp_sim_create_rank": ([ctypes.POINTER(SimConfig), ctypes.c_int, ctypes.c_int, _P, ctypes.POINTER(_P)],
                           ctypes.c_int),
    "rp_sim_shard_range": ([_P, _U32P, _U32P], ctypes.c_int),
    "rp_sim_local_counters": ([_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_sim_exchange_stats": ([_P, ctypes.POINTER(ctypes.c_double), _U64P, _U64P], ctypes.c_int),
    "rp_loop_create": ([ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "rp_loop_destroy": ([_P], ctypes.c_int),
    "rp_sim_create_rank_loop": ([ctypes.POINTER(SimConfig), _P, ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "rp_sim_exchange_shard_bytes": ([_P, _U64P, ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_sim_fail": ([_P, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
    "rp_sim_partition": ([_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
    "rp_sim_storm": ([_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
    "rp_sim_load_addresses": ([_P, _P, _P, ctypes.c_uint32], ctypes.c_int),
    "rp_sim_set_views": ([_P, ctypes.c_uint32, ctypes.c_uint32, _P, _P], ctypes.c_int),
    "rp_sim_join": ([_P, _P, _P, _P, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
    "rp_sim_round": ([_P, ctypes.c_int, ctypes.POINTER(RoundStats)], ctypes.c_int),
    "rp_sim_run": ([_P, ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "rp_sim_sync": ([_P], ctypes.c_int),
    "rp_sim_totals": ([_P, ctypes.POINTER(RoundStats)], ctypes.c_int),
    "rp_sim_rounds": ([_P, _U32P], ctypes.c_int),
    "rp_sim_counters": ([_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_sim_size": ([_P, _U32P], ctypes.c_int),
    "rp_sim_view_counts": ([_P, _P, _SZ], ctypes.c_int),
    "rp_sim_read_checksums": ([_P, _P, _SZ], ctypes.c_int),
    "rp_sim_read_view": ([_P, ctypes.c_uint32, _P, _P, _SZ], ctypes.c_int),
    "rp_sim_read_members": ([_P, ctypes.c_uint32, _P, _SZ, _U32P], ctypes.c_int),
    "rp_sim_read_changes": ([_P, ctypes.c_uint32, _P, ctypes.c_uint32, _U32P], ctypes.c_int),
    "rp_sim_node_info": ([_P, ctypes.c_uint32, _P], ctypes.c_int),
    "rp_sim_ring_lookup": ([_P, ctypes.c_uint32, _P, _SZ, _P], ctypes.c_int),
    "rp_sim_address": ([_P, ctypes.c_uint32, ctypes.c_char_p, _SZ], ctypes.c_int),
    "rp_sim_ping_body": ([_P, ctypes.c_uint32, _P, ctypes.c_uint32, _U32P, _U32P, ctypes.POINTER(ctypes.c_uint64)],
                         ctypes.c_int),
    "rp_sim_handle_ping": ([_P, ctypes.c_uint32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32, _P, ctypes.c_uint32,
                           _P, ctypes.c_uint32, _U32P, _U32P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_sim_update": ([_P, ctypes.c_uint32, _P, ctypes.c_uint32, _U32P], ctypes.c_int),
    "rp_sim_enable_timing": ([_P, ctypes.c_int], ctypes.c_int),
    "rp_sim_enable_timing_stages": ([_P, ctypes.c_uint32], ctypes.c_int),
    "rp_node_create": ([_P, _SZ, ctypes.c_uint64, ctypes.POINTER(_P)], ctypes.c_int),
    "rp_node_destroy": ([_P], ctypes.c_int),
    "rp_node_intern": ([_P, _P, _P, _SZ, _P], ctypes.c_int),
    "rp_node_address": ([_P, ctypes.c_uint32, ctypes.c_char_p, _SZ, ctypes.POINTER(_SZ)], ctypes.c_int),
    "rp_node_rng": ([_P, _U64P, _U64P], ctypes.c_int),
    "rp_membership_update": ([_P, _P, ctypes.c_uint32, ctypes.c_uint64, _P, _U32P, _U32P], ctypes.c_int),
    "rp_membership_set": ([_P, _P, ctypes.c_uint32, _P, _U32P, _U32P], ctypes.c_int),
    "rp_membership_checksum": ([_P, _U32P], ctypes.c_int),
    "rp_membership_checksum_string": ([_P, ctypes.c_char_p, _SZ, ctypes.POINTER(_SZ)], ctypes.c_int),
    "rp_membership_members": ([_P, _P, _P, _P, _SZ, _U32P], ctypes.c_int),
    "rp_membership_shuffle": ([_P], ctypes.c_int),
    "rp_membership_set_order": ([_P, _P, ctypes.c_uint32], ctypes.c_int),
    "rp_membership_random": ([_P, ctypes.c_uint32, _P], ctypes.c_int),
    "rp_membership_force": ([_P, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64], ctypes.c_int),
    "rp_dissemination_record": ([_P, _P, ctypes.c_uint32], ctypes.c_int),
    "rp_dissemination_issue": ([_P, ctypes.c_int32, _P, _SZ, _U32P], ctypes.c_int),
    "rp_dissemination_issue_as_receiver": ([_P, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.c_int32, _P, _SZ, _U32P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rp_dissemination_full_sync": ([_P, _P, _SZ, _U32P], ctypes.c_int),
    "rp_dissemination_clear": ([_P], ctypes.c_int),
    "rp_dissemination_changes": ([_P, _P, _SZ, _U32P], ctypes.c_int),
    "rp_sim_kernel_times": ([_P, _P, _P], ctypes.c_int),
    "rp_sim_side_ms": ([_P, _P], ctypes.c_int),
}

_lib = None


def lib():
    """Load libringpop_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RingpopError(-2, f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        variant = bool(os.environ.get("RINGPOP_HIP_LIB"))
        for name, (argt, rest) in SIGNATURES.items():
            if variant and not hasattr(L, name):
                continue  # an older build under A/B comparison: bind what it has
            f = getattr(L, name)
            f.argtypes = argt
            f.restype = rest
        _lib = L
    return _lib


def check(rc):
    if rc != RP_OK:
        raise RingpopError(rc, lib().rp_last_error().decode(errors="replace"))
    return rc


def ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)
