"""Trace record / replay.

A trace is everything needed to re-run a sequence of calls through any
implementation of the engine's surface — the HIP engine (raftstep.Engine),
the CPU oracle (oracle.Oracle, test infrastructure) or, where a Go toolchain
exists, a Go harness over the cgo shim — and to check it step by step:

  * the engine config (the raft_config fields),
  * the initial state (NewNode / post-election / an explicit canonical view),
  * the events: tick ranges (raft_tick) and handler batches
    (raft_append_entries_batch, raft_request_vote_batch, raft_group_ops_batch)
    with their request records exactly as they crossed the C-ABI,
  * what the recording implementation returned for each event (tick stats or
    response records) and the state digest after it (raft_state_digest).

Replay re-executes the events on another implementation and reports the
first event whose outputs or digest differ, with main.go nodelog lines
(main.go:399-401) of the groups whose per-group digests differ.

File format: one .npz (numpy, no pickles) holding a JSON "meta" document (as
uint8) plus one array per request/response record set.
"""
import json

import numpy as np

from . import abi

FORMAT = "raftstep-trace/1"
# (execution knobs that cannot change results are not part of a trace)
CONFIG_FIELDS = [name for name, _ in abi.Config._fields_
                 if name not in ("abi_version", "reserved", "ticks_per_launch", "debug_flags")]


def config_dict(cfg):
    return {k: int(getattr(cfg, k)) for k in CONFIG_FIELDS}


class TraceRecorder:
    """Forwards every call to `impl` and records it (and its outputs)."""

    # per-group digests are kept for traces up to this many groups, so that a
    # replay can name (and nodelog) the groups that diverge
    GROUP_DIGESTS_MAX = 4096

    def __init__(self, impl, digest_every=1):
        self.impl = impl
        self.meta = {"format": FORMAT, "config": config_dict(impl.cfg), "init": None, "events": []}
        self.arrays = {}
        self.digest_every = max(1, int(digest_every))

    @property
    def cfg(self):
        return self.impl.cfg

    # -- initial state --------------------------------------------------
    def init_new_nodes(self, tick0=0):
        self.impl.init_new_nodes(tick0)
        self.meta["init"] = {"kind": "new", "tick0": int(tick0), "digest": self._digest("init")}

    def init_steady(self, leader=0, tick0=0):
        self.impl.init_steady(leader, tick0)
        self.meta["init"] = {"kind": "steady", "leader": int(leader), "tick0": int(tick0),
                             "digest": self._digest("init")}

    def load_state(self, st):
        self.impl.load_state(st)
        for k in abi.STATE_FIELDS:
            self.arrays[f"init_{k}"] = np.ascontiguousarray(st[k])
        self.meta["init"] = {"kind": "state", "digest": self._digest("init")}

    # -- events -----------------------------------------------------------
    def _event(self, ev, outputs):
        i = len(self.meta["events"])
        for k, a in outputs.items():
            self.arrays[f"e{i}_{k}"] = a
        if (i + 1) % self.digest_every == 0:
            ev["digest"] = self._digest(f"e{i}")
        self.meta["events"].append(ev)

    def tick(self, first_tick, nticks=1, stats=True):
        s = self.impl.tick(first_tick, nticks, stats=True)
        self._event({"op": "tick", "first": int(first_tick), "n": int(nticks),
                     "stats": [int(x) for x in s]}, {})
        return s if stats else None

    def append_entries(self, now_tick, reqs, entries=None):
        out = self.impl.append_entries(now_tick, reqs, entries)
        i = len(self.meta["events"])
        self.arrays[f"e{i}_reqs"] = np.ascontiguousarray(reqs, dtype=abi.AE_REQ)
        self.arrays[f"e{i}_entries"] = (np.ascontiguousarray(entries, dtype=abi.LOG_ENTRY) if entries is not None
                                        else np.zeros(0, abi.LOG_ENTRY))
        self._event({"op": "ae", "now": int(now_tick)}, {"resp": out})
        return out

    def request_vote(self, now_tick, reqs):
        out = self.impl.request_vote(now_tick, reqs)
        i = len(self.meta["events"])
        self.arrays[f"e{i}_reqs"] = np.ascontiguousarray(reqs, dtype=abi.VOTE_REQ)
        self._event({"op": "vote", "now": int(now_tick)}, {"resp": out})
        return out

    def group_ops(self, now_tick, ops):
        out = self.impl.group_ops(now_tick, ops)
        i = len(self.meta["events"])
        self.arrays[f"e{i}_reqs"] = np.ascontiguousarray(ops, dtype=abi.GROUP_OP)
        self._event({"op": "ops", "now": int(now_tick)}, {"resp": out})
        return out

    def _digest(self, tag):
        per, tot = self.impl.state_digest()
        if len(per) <= self.GROUP_DIGESTS_MAX:
            self.arrays[f"{tag}_gdig"] = per
        return str(tot)   # u64 as a decimal string (JSON-safe)

    def save(self, path):
        meta = np.frombuffer(json.dumps(self.meta).encode(), dtype=np.uint8)
        np.savez_compressed(path, meta=meta, **self.arrays)


def load(path):
    """(meta dict, arrays dict) of a trace file."""
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(bytes(z["meta"]).decode())
        arrays = {k: z[k] for k in z.files if k != "meta"}
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} file")
    return meta, arrays


class Mismatch(AssertionError):
    pass


def replay(path, make_impl, nodelog_groups=4):
    """Re-run a trace on `make_impl(**config)` and check every recorded output
    and digest. Returns the implementation (for further inspection); raises
    Mismatch naming the first differing event, with nodelog lines of up to
    `nodelog_groups` groups whose digests differ."""
    meta, arrays = load(path)
    impl = make_impl(**meta["config"])
    init = meta["init"]
    if init["kind"] == "new":
        impl.init_new_nodes(init["tick0"])
    elif init["kind"] == "steady":
        impl.init_steady(init["leader"], init["tick0"])
    else:
        impl.load_state({k: arrays[f"init_{k}"] for k in abi.STATE_FIELDS})
    _check_digest(impl, init["digest"], arrays.get("init_gdig"), "initial state", nodelog_groups)
    for i, ev in enumerate(meta["events"]):
        op = ev["op"]
        what = f"event {i} ({op})"
        if op == "tick":
            s = impl.tick(ev["first"], ev["n"], stats=True)
            if [int(x) for x in s] != ev["stats"]:
                raise Mismatch(f"{what}: stats {list(map(int, s))} != recorded {ev['stats']}")
        else:
            reqs = arrays[f"e{i}_reqs"]
            if op == "ae":
                out = impl.append_entries(ev["now"], reqs, arrays[f"e{i}_entries"])
            elif op == "vote":
                out = impl.request_vote(ev["now"], reqs)
            elif op == "ops":
                out = impl.group_ops(ev["now"], reqs)
            else:
                raise ValueError(f"{path}: unknown event op {op!r}")
            want = arrays[f"e{i}_resp"]
            if out.tobytes() != want.tobytes():
                bad = np.nonzero(out != want)[0][:8].tolist()
                raise Mismatch(f"{what}: responses differ at records {bad}")
        if "digest" in ev:
            _check_digest(impl, ev["digest"], arrays.get(f"e{i}_gdig"), what, nodelog_groups)
    return impl


def _check_digest(impl, want, want_per, what, nodelog_groups):
    per, tot = impl.state_digest()
    if str(tot) == want:
        return
    msg = f"{what}: state digest {tot} != recorded {want}"
    if want_per is not None:
        bad = np.nonzero(per != want_per)[0]
        msg += f"; {len(bad)} groups differ, first {bad[:8].tolist()}:\n"
        msg += nodelog_dump(impl, bad[:nodelog_groups])
    raise Mismatch(msg)


def nodelog_dump(impl, groups):
    """main.go-format lines of the given groups (for diffing implementations)."""
    return "".join(f"# group {g}\n" + impl.nodelog(int(g)) for g in groups)
