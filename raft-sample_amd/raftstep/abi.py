"""ctypes mirror of include/raftstep.h (the C-ABI boundary).

Record layouts are declared twice — as ctypes Structures for scalar calls and
as numpy structured dtypes for batches — and checked against each other at
import time, so a header change that is not mirrored here fails loudly.
"""
import ctypes as C

import numpy as np

RAFT_ABI_VERSION = 6
RAFT_MAX_REPLICAS = 8

FOLLOWER, CANDIDATE, LEADER = 0, 1, 2
SEM_REF, SEM_RAFT = 0, 1
CLIENT_TRACE, CLIENT_STAGED = 0, 1   # raft_config.client_source (include/raftstep.h)
ROLE_NAMES = {FOLLOWER: "follower", CANDIDATE: "candidate", LEADER: "leader"}  # main.go:51-57

F_NONE, F_PANIC_GETLOG, F_DEADLOCK_VRES, F_DEADLOCK_LEADER_VREQ, F_RING_EVICTED, F_OVERFLOW = range(6)

STAT_NAMES = ("committed", "elections_won", "term_bumps", "ae_ok", "ae_fail",
              "votes_granted", "faults", "leader_groups")
NSTATS = len(STAT_NAMES)

OP_CLIENT_APPEND, OP_LEADER_ROUND, OP_CANDIDATE_ROUND, OP_TIMEOUT, OP_LEADER_COMMIT = 1, 2, 3, 4, 5

RAFT_EINVAL, RAFT_ENOMEM, RAFT_ERANGE, RAFT_ENODEV = -22, -12, -34, -19
RAFT_EINTERNAL = -3000

DEBUG_ALLOW_WRONG_RESULTS = 1   # raft_config.debug_flags: accept RAFTSTEP_DIAG_LEAN (timing only, results wrong)

# raft_diag_read counters (include/raftstep.h enum raft_diag_counter)
DIAG_COUNTERS = 72
DIAG = {
    "lean_lanes": 10, "lean_skipped": 0, "lean_ssync": 18, "lean_lxs": 19, "lean_three_seg": 20,
    "lean_lxs_whole_row": 21, "lean_hwx": 22, "lean_passed": 23, "lean_forced": 24, "lean_switch": 5,
    "lean_sxs": 25, "lean_sxs_stale_in_row": 26, "list_sxs_materialised": 61, "list_sxs_entered": 62,
    "list_stale_moved": 63, "lean_sxs_vx": 27, "list_return_vx": 28, "list_lxs_vx": 29,
    "lean_sh": 30, "list_sh_copied": 31, "list_sh_entries": 1, "list_lag_catchup": 6, "list_sh_kept": 7,
    "list_lanes": 42, "list_deferred": 33, "list_isolation": 34, "list_switch": 37, "list_quiet": 48,
    "list_isolated_leader": 49, "list_ssync": 50, "list_election": 51, "list_first_round": 52,
    "list_return": 53, "list_return_trunc": 54, "list_stale": 55, "list_hwx": 56, "list_three_seg": 57,
    "list_isolated_replica": 58, "list_timer_fire": 59, "list_window_start": 60,
    "ticks": 64, "ticks_list_skipped": 65, "general_launches": 66,
}


class Config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32), ("replicas", C.c_uint32),
        ("groups", C.c_uint64), ("group_base", C.c_uint64),
        ("ring_depth", C.c_uint32), ("entries_per_tick", C.c_uint32),
        ("client_period", C.c_uint32), ("semantics", C.c_uint32),
        ("seed", C.c_uint64),
        ("tick_seconds", C.c_int32),
        ("follower_timeout_min", C.c_int32), ("follower_timeout_span", C.c_int32),
        ("candidate_timeout_min", C.c_int32), ("candidate_timeout_span", C.c_int32),
        ("isolate_per_65536", C.c_uint32), ("isolate_min_ticks", C.c_uint32),
        ("isolate_max_ticks", C.c_uint32),
        ("device", C.c_int32),
        ("payload_crc", C.c_uint32), ("corrupt_per_65536", C.c_uint32),
        ("isolate_leader", C.c_uint32),
        ("ticks_per_launch", C.c_uint32), ("debug_flags", C.c_uint32),
        ("client_source", C.c_uint32),
        ("reserved", C.c_uint32 * 2),
    ]


def default_config(**kw):
    """Defaults of raft_config_default() (main.go's constants), overridden by kw."""
    c = Config()
    c.abi_version = RAFT_ABI_VERSION
    c.replicas = 3            # main.go:81
    c.groups = 1
    c.ring_depth = 32
    c.entries_per_tick = 1
    c.client_period = 5       # one write per 10 s (main.go:89) at 2 s per tick
    c.semantics = 0
    c.seed = 0x5EED0001
    c.tick_seconds = 2        # main.go:394
    c.follower_timeout_min, c.follower_timeout_span = 10, 20    # main.go:114
    c.candidate_timeout_min, c.candidate_timeout_span = 10, 4   # main.go:194
    c.isolate_per_65536 = 0
    c.isolate_min_ticks, c.isolate_max_ticks = 8, 32
    c.device = 0
    c.payload_crc = 0
    c.corrupt_per_65536 = 0
    c.isolate_leader = 0
    c.ticks_per_launch = 1    # one tick per launch
    c.debug_flags = 0
    c.client_source = CLIENT_TRACE   # values from the trace RNG (main.go:92's rand.Int())
    for k, v in kw.items():
        if not hasattr(c, k):
            raise TypeError(f"unknown config field {k!r}")
        setattr(c, k, v)
    return c


class TickStats(C.Structure):
    _fields_ = [("v", C.c_int64 * NSTATS)]


class StateView(C.Structure):
    _fields_ = [
        ("role", C.c_void_p), ("voted", C.c_void_p), ("term", C.c_void_p),
        ("last", C.c_void_p), ("commit", C.c_void_p), ("deadline", C.c_void_p),
        ("timeout", C.c_void_p), ("match", C.c_void_p), ("fault", C.c_void_p),
        ("log_term", C.c_void_p), ("log_value", C.c_void_p), ("log_crc", C.c_void_p),
        ("next", C.c_void_p), ("hwm", C.c_void_p), ("iso_victim", C.c_void_p),
    ]


STATE_FIELDS = ("role", "voted", "term", "last", "commit", "deadline", "timeout",
                "match", "fault", "log_term", "log_value", "log_crc", "next", "hwm", "iso_victim")


def state_shapes(groups, replicas, ring_depth):
    G, R, K = groups, replicas, ring_depth
    return {
        "role": ((G, R), np.uint8), "voted": ((G, R), np.uint8),
        "term": ((G, R), np.int32), "last": ((G, R), np.int32),
        "commit": ((G, R), np.int32), "deadline": ((G, R), np.int32),
        "timeout": ((G, R), np.int32), "match": ((G, R, R), np.int32),
        "fault": ((G,), np.uint8), "log_term": ((G, R, K), np.int32),
        "log_value": ((G, R, K), np.int64), "log_crc": ((G, R, K), np.uint32),
        "next": ((G, R, R), np.int32), "hwm": ((G, R), np.int32),
        "iso_victim": ((G,), np.uint8),
    }


def empty_state(groups, replicas, ring_depth):
    return {k: np.zeros(s, d) for k, (s, d) in state_shapes(groups, replicas, ring_depth).items()}


OPTIONAL_ON_LOAD = ("log_crc", "next", "hwm", "iso_victim")   # raft_load_state: NULL derives them (raftstep.h)


def coerce_state(state, groups, replicas, ring_depth):
    """Canonical view arrays for raft_load_state: each field converted to its
    C type and checked against its shape (a wrong dtype would be read as
    garbage, a short array past its end); optional fields may be absent."""
    out = {}
    for k, (shape, dt) in state_shapes(groups, replicas, ring_depth).items():
        a = state.get(k)
        if a is None:
            if k in OPTIONAL_ON_LOAD:
                continue
            raise KeyError(f"state field {k!r} is required")
        a = np.asarray(a)
        if a.dtype.kind not in "iub":
            raise TypeError(f"state field {k!r}: integer array expected, got {a.dtype}")
        if a.shape != shape:
            raise ValueError(f"state field {k!r}: shape {a.shape}, expected {shape}")
        c = np.ascontiguousarray(a, dtype=dt)
        if not np.array_equal(c, a):
            raise ValueError(f"state field {k!r}: values do not fit {np.dtype(dt).name}")
        out[k] = c
    return out


def make_view(state):
    v = StateView()
    for k in STATE_FIELDS:
        a = state.get(k)
        if a is not None:
            assert a.flags["C_CONTIGUOUS"], k
            setattr(v, k, a.ctypes.data)
    return v


# batch records (numpy, C layout)
AE_REQ = np.dtype([("group", "<u8"), ("to", "<u4"), ("leader_id", "<u4"), ("term", "<i8"),
                   ("prev_log_index", "<i8"), ("prev_log_term", "<i8"), ("leader_commit", "<i8"),
                   ("entries_offset", "<u8"), ("n_entries", "<u8")], align=True)
AE_RESP = np.dtype([("term", "<i8"), ("match_index", "<i8"), ("success", "<i4"), ("fault", "<i4")],
                   align=True)
LOG_ENTRY = np.dtype([("term", "<i8"), ("value", "<i8")], align=True)
VOTE_REQ = np.dtype([("group", "<u8"), ("to", "<u4"), ("candidate_id", "<u4"), ("term", "<i8"),
                     ("last_log_index", "<i8"), ("last_log_term", "<i8")], align=True)
VOTE_RESP = np.dtype([("term", "<i8"), ("vote_granted", "<i4"), ("fault", "<i4")], align=True)
GROUP_OP = np.dtype([("group", "<u8"), ("replica", "<u4"), ("kind", "<u4"), ("arg", "<i8")], align=True)
OP_RESULT = np.dtype([("status", "<i4"), ("fault", "<i4"), ("value", "<i8")], align=True)

assert AE_REQ.itemsize == 64 and AE_RESP.itemsize == 24 and LOG_ENTRY.itemsize == 16
assert VOTE_REQ.itemsize == 40 and VOTE_RESP.itemsize == 16
assert GROUP_OP.itemsize == 24 and OP_RESULT.itemsize == 16
assert C.sizeof(Config) == 120, C.sizeof(Config)

# exported symbols of libraftstep.so (the C-ABI), with ctypes signatures
P = C.c_void_p
SIGNATURES = {
    "raft_config_default": (None, [P]),
    "raft_engine_create": (C.c_int, [P, C.POINTER(C.c_void_p)]),
    "raft_engine_destroy": (C.c_int, [P]),
    "raft_last_error": (C.c_char_p, []),
    "raft_engine_info": (C.c_int, [P, P, P]),
    "raft_engine_features": (C.c_int, [P, P]),
    "raft_init_new_nodes": (C.c_int, [P, C.c_int64]),
    "raft_init_steady": (C.c_int, [P, C.c_int32, C.c_int64]),
    "raft_load_state": (C.c_int, [P, P]),
    "raft_store_state": (C.c_int, [P, P]),
    "raft_store_state_range": (C.c_int, [P, C.c_uint64, C.c_uint64, P]),
    "raft_tick": (C.c_int, [P, C.c_int64, C.c_uint32, P]),
    "raft_stage_values": (C.c_int, [P, C.c_int64, C.c_uint32, P]),
    "raft_sync": (C.c_int, [P]),
    "raft_tick_records": (C.c_int, [P, C.c_uint32, P]),
    "raft_comm_info": (C.c_int, [P, P, P, P]),
    "raft_append_entries_batch": (C.c_int, [P, C.c_int64, P, C.c_size_t, P, C.c_size_t, P]),
    "raft_request_vote_batch": (C.c_int, [P, C.c_int64, P, C.c_size_t, P]),
    "raft_group_ops_batch": (C.c_int, [P, C.c_int64, P, C.c_size_t, P]),
    "raft_comm_unique_id": (C.c_int, [P]),
    "raft_comm_init": (C.c_int, [P, C.c_int, C.c_int, P]),
    "raft_comm_allreduce_stats": (C.c_int, [P, P]),
    "raft_profile_enable": (C.c_int, [P, C.c_int]),
    "raft_profile_read": (C.c_int, [P, P, P]),
    "raft_state_digest": (C.c_int, [P, P, P]),
    "raft_nodelog": (C.c_int, [P, C.c_uint64, C.c_char_p, C.c_size_t]),
    "raft_checkpoint_save": (C.c_int, [P, C.c_char_p]),
    "raft_checkpoint_load": (C.c_int, [P, C.c_char_p]),
    "raft_diag_enable": (C.c_int, [P, C.c_int]),
    "raft_diag_read": (C.c_int, [P, P, C.c_uint32]),
    "raft_debug_force_pass": (C.c_int, [P, C.c_int64]),
    "raft_debug_diag_mode": (C.c_int, [P, C.c_uint32]),
    "raft_stream_probe": (C.c_int, [C.c_int, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                                    C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "raft_debug_group_words": (C.c_int, [P, C.c_uint64, P, C.c_uint32]),
}


# measurement / diagnostics entry points added in round 5: an older build
# loaded through RAFTSTEP_LIB (A/B runs) may lack them
OPTIONAL = ("raft_debug_diag_mode", "raft_stream_probe", "raft_engine_features")
FEATURE_SHARED_ENTRIES, FEATURE_VIRTUAL_SUFFIXES = 1, 2   # raft_engine_features (include/raftstep.h)
PROBE_PLAIN_RING, PROBE_NT_RECORD, PROBE_NO_HEARTBEAT = 1, 2, 4   # raft_stream_probe flags


def bind(lib):
    for name, (res, args) in SIGNATURES.items():
        if name in OPTIONAL and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib
