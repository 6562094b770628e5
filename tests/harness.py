"""Shared helpers for parity tests: build canonical states by hand, compare
states field by field, hash states per tick, and build handler batches.
Used with both the oracle (CPU) and the engine (GPU): both expose the same
methods (init_*, load_state, store_state, tick, append_entries,
request_vote, group_ops)."""
import hashlib

import numpy as np

from raftstep import abi

F, C, L = abi.FOLLOWER, abi.CANDIDATE, abi.LEADER


def node(role=F, term=0, voted=0, log=(), commit=0, deadline=1000, timeout=20, match=None):
    """One replica's state; log is a list of (term, value) = Node.Log (main.go:21)."""
    return dict(role=role, term=term, voted=voted, log=list(log), commit=commit,
                deadline=deadline, timeout=timeout, match=match)


def build_state(groups_nodes, R, K, faults=None):
    """groups_nodes: list (per group) of list (per replica) of node() dicts."""
    G = len(groups_nodes)
    st = abi.empty_state(G, R, K)
    for g, nodes in enumerate(groups_nodes):
        assert len(nodes) == R
        for r, n in enumerate(nodes):
            st["role"][g, r] = n["role"]
            st["voted"][g, r] = n["voted"]
            st["term"][g, r] = n["term"]
            st["last"][g, r] = len(n["log"])
            st["commit"][g, r] = n["commit"]
            st["deadline"][g, r] = n["deadline"]
            st["timeout"][g, r] = n["timeout"]
            if n["role"] == L:
                m = n["match"] or [0] * R
                for p in range(R):
                    st["match"][g, r, p] = 0 if p == r else m[p]
            last = len(n["log"])
            for i in range(max(1, last - K + 1), last + 1):
                t, v = n["log"][i - 1]
                st["log_term"][g, r, (i - 1) % K] = t
                st["log_value"][g, r, (i - 1) % K] = v
        if faults is not None:
            st["fault"][g] = faults[g]
    return st


def log_of(st, g, r, K):
    """The visible tail of replica r's log as a list of (term, value)."""
    last = int(st["last"][g, r])
    return [(int(st["log_term"][g, r, (i - 1) % K]), int(st["log_value"][g, r, (i - 1) % K]))
            for i in range(max(1, last - K + 1), last + 1)]


def diff_states(a, b, fields=abi.STATE_FIELDS, limit=8):
    """Human-readable list of mismatches (empty when equal)."""
    out = []
    for k in fields:
        if k not in a or k not in b:
            continue
        x, y = np.asarray(a[k]), np.asarray(b[k])
        if x.shape != y.shape:
            out.append(f"{k}: shape {x.shape} vs {y.shape}")
            continue
        bad = np.argwhere(x != y)
        for idx in bad[:limit]:
            t = tuple(int(i) for i in idx)
            out.append(f"{k}{list(t)}: {x[t]} != {y[t]}")
        if len(bad) > limit:
            out.append(f"{k}: ... {len(bad)} mismatches")
    return out


def assert_same_state(a, b, what=""):
    d = diff_states(a, b)
    assert not d, f"state mismatch {what}:\n" + "\n".join(d)


def state_hash(st):
    h = hashlib.sha256()
    for k in abi.STATE_FIELDS:
        if k in st:
            h.update(k.encode())
            h.update(np.ascontiguousarray(st[k]).tobytes())
    return h.hexdigest()


def group_hashes(st, raft_fields=False):
    """Per-group digest (uint64) of every field — for per-tick trace diffs
    (log_crc / iso_victim only when present and non-zero, i.e. with
    payload_crc / leader-isolation mode on;
    next/hwm only with raft_fields: in REF mode they are derived from
    match/last, and the committed golden digests predate them)."""
    G = st["fault"].shape[0]
    acc = np.zeros(G, dtype=np.uint64)
    mult = np.uint64(0x100000001B3)
    with np.errstate(over="ignore"):
        for k in abi.STATE_FIELDS:
            if k in ("next", "hwm") and not raft_fields:
                continue
            if k not in st or (k in ("log_crc", "iso_victim") and not st[k].any()):
                continue
            a = np.ascontiguousarray(st[k]).reshape(G, -1).astype(np.int64).view(np.uint64)
            for j in range(a.shape[1]):
                acc = (acc ^ a[:, j]) * mult
    return acc


def ae_reqs(items):
    """items: list of dicts(group, to, term, prev_log_index, prev_log_term, leader_commit, logs=[(t,v)])."""
    reqs = np.zeros(len(items), abi.AE_REQ)
    ents = []
    for i, it in enumerate(items):
        logs = it.get("logs", [])
        reqs[i]["group"] = it.get("group", i)
        reqs[i]["to"] = it["to"]
        reqs[i]["leader_id"] = it.get("leader_id", 0)
        reqs[i]["term"] = it["term"]
        reqs[i]["prev_log_index"] = it.get("prev_log_index", 0)
        reqs[i]["prev_log_term"] = it.get("prev_log_term", 0)
        reqs[i]["leader_commit"] = it.get("leader_commit", 0)
        reqs[i]["entries_offset"] = len(ents)
        reqs[i]["n_entries"] = len(logs)
        ents.extend(logs)
    e = np.zeros(len(ents), abi.LOG_ENTRY)
    for i, (t, v) in enumerate(ents):
        e[i]["term"], e[i]["value"] = t, v
    return reqs, e


def vote_reqs(items):
    reqs = np.zeros(len(items), abi.VOTE_REQ)
    for i, it in enumerate(items):
        reqs[i]["group"] = it.get("group", i)
        reqs[i]["to"] = it["to"]
        reqs[i]["candidate_id"] = it.get("candidate_id", 0)
        reqs[i]["term"] = it["term"]
    return reqs


def ops(items):
    o = np.zeros(len(items), abi.GROUP_OP)
    for i, it in enumerate(items):
        o[i]["group"] = it.get("group", i)
        o[i]["replica"] = it["replica"]
        o[i]["kind"] = it["kind"]
        o[i]["arg"] = it.get("arg", 0)
    return o


def crc32c(data):
    """Bitwise CRC32C (Castagnoli, reflected 0x82F63B78) — independent of both implementations."""
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 & -(c & 1))
    return c ^ 0xFFFFFFFF


def entry_crc(term, value):
    """EXT stamp of a log entry: CRC32C(Term as 4 B LE || Value as 8 B LE)."""
    return crc32c((int(term) & 0xFFFFFFFF).to_bytes(4, "little") + (int(value) & (2**64 - 1)).to_bytes(8, "little"))


def stamp_crcs(st):
    """Fill log_crc with the stamps of the visible ring entries."""
    G, R, K = st["log_term"].shape
    st["log_crc"][:] = 0
    for g in range(G):
        for r in range(R):
            last = int(st["last"][g, r])
            for i in range(max(1, last - K + 1), last + 1):
                s = (i - 1) % K
                st["log_crc"][g, r, s] = entry_crc(int(st["log_term"][g, r, s]), int(st["log_value"][g, r, s]))
    return st


def random_state(rng, G, R, K, max_term=6, max_log=12):
    """Random but well-formed canonical state (LastApplied == len(Log)), used
    to drive both implementations through rarely reached handler branches."""
    st = abi.empty_state(G, R, K)
    st["role"][:] = rng.integers(0, 3, (G, R))
    st["voted"][:] = rng.integers(0, 2, (G, R))
    st["term"][:] = rng.integers(0, max_term, (G, R))
    st["last"][:] = rng.integers(0, max_log + 1, (G, R))
    st["commit"][:] = rng.integers(0, max_log + 2, (G, R))
    st["timeout"][:] = rng.integers(10, 30, (G, R))
    st["deadline"][:] = rng.integers(0, 60, (G, R))
    for g in range(G):
        for r in range(R):
            last = int(st["last"][g, r])
            for i in range(max(1, last - K + 1), last + 1):
                st["log_term"][g, r, (i - 1) % K] = rng.integers(0, max_term)
                st["log_value"][g, r, (i - 1) % K] = rng.integers(0, 1 << 62)
            if st["role"][g, r] == L:
                for p in range(R):
                    if p != r:
                        st["match"][g, r, p] = rng.integers(0, max_log + 2)
    return st


def random_events(impl, rng, n_events, t0=0):
    """Drive `impl` (engine, oracle or a trace.TraceRecorder over one) through a
    random mix of tick ranges and handler batches; returns the next tick."""
    G, R = impl.cfg.groups, impl.cfg.replicas
    t = t0
    for _ in range(n_events):
        kind = int(rng.integers(0, 5))
        groups = rng.permutation(G)[: max(1, G // 3)]
        if kind <= 1:
            k = int(rng.integers(1, 6))
            impl.tick(t, k)
            t += k
        elif kind == 2:
            items = [dict(group=int(g), to=int(rng.integers(0, R)), term=int(rng.integers(0, 6)),
                          prev_log_index=int(rng.integers(0, 8)), prev_log_term=int(rng.integers(0, 6)),
                          leader_commit=int(rng.integers(0, 10)),
                          logs=[(int(rng.integers(0, 6)), int(rng.integers(0, 1 << 62)))
                                for _ in range(int(rng.integers(0, 5)))]) for g in groups]
            reqs, ents = ae_reqs(items)
            impl.append_entries(t, reqs, ents)
        elif kind == 3:
            impl.request_vote(t, vote_reqs([dict(group=int(g), to=int(rng.integers(0, R)),
                                                 term=int(rng.integers(0, 8)),
                                                 candidate_id=int(rng.integers(0, R))) for g in groups]))
        else:
            impl.group_ops(t, ops([dict(group=int(g), replica=int(rng.integers(0, R)), kind=int(rng.integers(1, 6)),
                                        arg=int(rng.integers(0, 1 << 62))) for g in groups]))
    return t
