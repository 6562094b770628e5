"""Python handle over libraftstep.so (the HIP engine), through the C-ABI only.

There is deliberately no CPU fallback: if the library or a GPU is missing
the constructor raises. The CPU restatement lives in oracle/ and is test
infrastructure, never imported from here.
"""
import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RAFTSTEP_LIB") or os.path.normpath(os.path.join(_HERE, "..", "lib", "libraftstep.so"))   # env: A/B of another build
_lib = None


class RaftError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"raftstep error {code}: {msg}")
        self.code = code


def load_library(path=None):
    """Load and bind libraftstep.so; raises if it is missing (no fallback)."""
    global _lib
    if _lib is None or path:
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RaftError(-2, f"{p} not built (run __graft_entry__.build() or make -C raft-sample_amd/csrc)")
        _lib = abi.bind(C.CDLL(p))
    return _lib


def _check(rc):
    if rc != 0:
        raise RaftError(rc, load_library().raft_last_error().decode(errors="replace"))


def stream_probe(device=0, replicas=5, elems=1 << 24, reps=10, heartbeat=True, flags=0):
    """The steady lean kernel's byte mix on fresh buffers (raft_stream_probe):
    (us per pass, bytes per pass). heartbeat=False: without the heartbeat
    store (a group in shared form; abi.PROBE_NO_HEARTBEAT). `flags`: further
    abi.PROBE_* bits (store policies, A/B)."""
    lib = load_library()
    us, by = C.c_double(), C.c_double()
    f = int(flags) | (0 if heartbeat else abi.PROBE_NO_HEARTBEAT)
    _check(lib.raft_stream_probe(int(device), int(replicas), int(elems), int(reps), f, C.byref(us), C.byref(by)))
    return us.value, by.value


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


class Engine:
    """One engine = the groups of one GPU (config.group_base.. +groups)."""

    def __init__(self, cfg=None, **kw):
        self.lib = load_library()
        self.cfg = cfg if cfg is not None else abi.default_config(**kw)
        if cfg is not None and kw:
            for k, v in kw.items():
                setattr(self.cfg, k, v)
        h = C.c_void_p()
        _check(self.lib.raft_engine_create(C.byref(self.cfg), C.byref(h)))
        self.h = h

    # -- lifecycle -----------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.raft_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def groups(self):
        return self.cfg.groups

    @property
    def replicas(self):
        return self.cfg.replicas

    def device_bytes(self):
        b = C.c_uint64()
        _check(self.lib.raft_engine_info(self.h, None, C.byref(b)))
        return b.value

    def features(self):
        """Storage forms in use (raft_engine_features): shared_entries,
        virtual_suffixes. Results are identical either way."""
        f = C.c_uint32()
        if hasattr(self.lib, "raft_engine_features"):
            _check(self.lib.raft_engine_features(self.h, C.byref(f)))
        return {"shared_entries": bool(f.value & abi.FEATURE_SHARED_ENTRIES),
                "virtual_suffixes": bool(f.value & abi.FEATURE_VIRTUAL_SUFFIXES)}

    # -- state ---------------------------------------------------------
    def init_new_nodes(self, tick0=0):
        _check(self.lib.raft_init_new_nodes(self.h, tick0))

    def init_steady(self, leader=0, tick0=0):
        _check(self.lib.raft_init_steady(self.h, leader, tick0))

    def store_state(self, logs=True):
        st = abi.empty_state(self.cfg.groups, self.cfg.replicas, self.cfg.ring_depth)
        if not logs:
            for k in ("log_term", "log_value", "log_crc"):
                st.pop(k)
        v = abi.make_view(st)
        _check(self.lib.raft_store_state(self.h, C.byref(v)))
        return st

    def store_state_range(self, first_group, n_groups, logs=True):
        """Canonical view of groups [first_group, first_group + n_groups) only (local indices)."""
        st = abi.empty_state(n_groups, self.cfg.replicas, self.cfg.ring_depth)
        if not logs:
            for k in ("log_term", "log_value", "log_crc"):
                st.pop(k)
        v = abi.make_view(st)
        _check(self.lib.raft_store_state_range(self.h, first_group, n_groups, C.byref(v)))
        return st

    def load_state(self, st):
        st = abi.coerce_state(st, self.cfg.groups, self.cfg.replicas, self.cfg.ring_depth)
        v = abi.make_view(st)
        _check(self.lib.raft_load_state(self.h, C.byref(v)))

    # -- audit ---------------------------------------------------------
    def state_digest(self):
        """(per-group digests u64[G], wrapping sum), computed on the device."""
        per = np.zeros(self.cfg.groups, np.uint64)
        tot = C.c_uint64()
        _check(self.lib.raft_state_digest(self.h, _ptr(per), C.byref(tot)))
        return per, tot.value

    def nodelog(self, group):
        """main.go nodelog lines (main.go:399-401) of every replica of `group`."""
        buf = C.create_string_buffer(64 * (self.cfg.replicas + 1))
        n = self.lib.raft_nodelog(self.h, group, buf, len(buf))
        if n < 0:
            _check(n)
        return buf.value.decode()

    def save_checkpoint(self, path):
        _check(self.lib.raft_checkpoint_save(self.h, os.fsencode(path)))

    def load_checkpoint(self, path):
        _check(self.lib.raft_checkpoint_load(self.h, os.fsencode(path)))

    # -- the fused tick ------------------------------------------------
    def tick(self, first_tick, nticks=1, stats=True):
        if stats:
            s = abi.TickStats()
            _check(self.lib.raft_tick(self.h, first_tick, nticks, C.byref(s)))
            return np.array(s.v, dtype=np.int64)
        _check(self.lib.raft_tick(self.h, first_tick, nticks, None))
        return None

    def stage_values(self, first_tick, values):
        """RAFT_CLIENT_STAGED: copy the client values of ticks first_tick ..
        first_tick + len(values) - 1 into HBM; values[t][e][g] int64
        (raft_stage_values: [nticks][E][G])."""
        v = np.ascontiguousarray(values, dtype=np.int64)
        if v.ndim != 3 or v.shape[1:] != (self.cfg.entries_per_tick, self.cfg.groups):
            raise ValueError(f"staged values: shape {v.shape}, expected (nticks, {self.cfg.entries_per_tick}, "
                             f"{self.cfg.groups})")
        _check(self.lib.raft_stage_values(self.h, int(first_tick), v.shape[0], _ptr(v)))

    def tick_records(self, nticks):
        """Per-tick stats [nticks][8] of the last tick(stats=True) call (device-reduced,
        summed over GPUs with a communicator)."""
        recs = (abi.TickStats * nticks)()
        _check(self.lib.raft_tick_records(self.h, nticks, recs))
        return np.array([list(r.v) for r in recs], dtype=np.int64).reshape(nticks, abi.NSTATS)

    def sync(self):
        _check(self.lib.raft_sync(self.h))

    # -- handler batches -----------------------------------------------
    def append_entries(self, now_tick, reqs, entries=None):
        reqs = np.ascontiguousarray(reqs, dtype=abi.AE_REQ)
        ents = np.ascontiguousarray(entries if entries is not None else np.zeros(0, abi.LOG_ENTRY),
                                    dtype=abi.LOG_ENTRY)
        out = np.zeros(len(reqs), abi.AE_RESP)
        _check(self.lib.raft_append_entries_batch(self.h, now_tick, _ptr(reqs), len(reqs), _ptr(ents),
                                                  len(ents), _ptr(out)))
        return out

    def request_vote(self, now_tick, reqs):
        reqs = np.ascontiguousarray(reqs, dtype=abi.VOTE_REQ)
        out = np.zeros(len(reqs), abi.VOTE_RESP)
        _check(self.lib.raft_request_vote_batch(self.h, now_tick, _ptr(reqs), len(reqs), _ptr(out)))
        return out

    def group_ops(self, now_tick, ops):
        ops = np.ascontiguousarray(ops, dtype=abi.GROUP_OP)
        out = np.zeros(len(ops), abi.OP_RESULT)
        _check(self.lib.raft_group_ops_batch(self.h, now_tick, _ptr(ops), len(ops), _ptr(out)))
        return out

    # -- multi-GPU -----------------------------------------------------
    @staticmethod
    def comm_unique_id():
        buf = (C.c_uint8 * 128)()
        _check(load_library().raft_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _check(self.lib.raft_comm_init(self.h, nranks, rank, buf))

    def comm_info(self):
        """(nranks, rank, allreduces issued) as RCCL reports them (1, 0, n without a communicator)."""
        n, r, k = C.c_int32(), C.c_int32(), C.c_uint64()
        _check(self.lib.raft_comm_info(self.h, C.byref(n), C.byref(r), C.byref(k)))
        return n.value, r.value, k.value

    def allreduce_stats(self, stats):
        s = abi.TickStats()
        for i, x in enumerate(stats):
            s.v[i] = int(x)
        _check(self.lib.raft_comm_allreduce_stats(self.h, C.byref(s)))
        return np.array(s.v, dtype=np.int64)

    # -- instrumentation -----------------------------------------------
    def profile(self, mode=1):
        """0 off, 1 per-dispatch events on the steady-state kernel, 2 one event pair per tick()
        call, 3 per-dispatch events on the two-pass plan's list kernel."""
        _check(self.lib.raft_profile_enable(self.h, int(mode)))

    def profile_read(self):
        ms, n = C.c_double(), C.c_uint64()
        _check(self.lib.raft_profile_read(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    # -- diagnostics ---------------------------------------------------
    def diag_enable(self, on=True):
        """Zero and start (or stop) the tick-class counters (raft_diag_enable)."""
        _check(self.lib.raft_diag_enable(self.h, int(bool(on))))

    def diag_read(self):
        """{class name: lanes} since the last read (abi.DIAG names; raft_diag_read), then zeroed."""
        buf = (C.c_uint64 * abi.DIAG_COUNTERS)()
        _check(self.lib.raft_diag_read(self.h, buf, abi.DIAG_COUNTERS))
        return {k: int(buf[i]) for k, i in abi.DIAG.items()}

    def debug_group_words(self, group):
        """Raw per-group words (gmeta, giso, hb, gss[4], glx[2], grot, grota, gsb, grotb, gsb2)."""
        buf = (C.c_int32 * 14)()
        _check(self.lib.raft_debug_group_words(self.h, int(group), buf, 14))
        names = ("meta", "giso", "hb", "ss_last", "ss_term", "ss_cl", "ss_cf", "lx_k", "lx_dl", "rot", "rota", "sb",
                 "rotb", "sb2")
        return dict(zip(names, list(buf)))

    def debug_diag_mode(self, mode):
        """Timing diagnostics (results wrong while non-zero; engine created with
        debug_flags=abi.DEBUG_ALLOW_WRONG_RESULTS)."""
        _check(self.lib.raft_debug_diag_mode(self.h, int(mode)))

    def debug_force_pass(self, group):
        """Test knob: the lean kernel passes `group` (-1: none) to the list kernel."""
        _check(self.lib.raft_debug_force_pass(self.h, int(group)))
