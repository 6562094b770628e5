"""The EXT RAFT-paper semantics mode (semantics=1) on the HIP engine: the
hand-derived KATs of tests/kat_raft.py, random handler batches on random
well-formed RAFT states, and whole tick traces with isolation churn, all
bit-exact against the oracle's r_* restatement."""
import numpy as np
import pytest

import harness as H
import kat_raft
from raftstep import Engine, abi

pytestmark = pytest.mark.gpu


def make_engine(kw):
    return Engine(**kw)


@pytest.mark.parametrize("case", kat_raft.ALL, ids=lambda f: f.__name__)
def test_engine_raft_kat(case):
    case(make_engine)


def pair(**kw):
    import oracle
    kw = dict(kw, semantics=abi.SEM_RAFT)
    return Engine(**kw), oracle.Oracle(**kw)


def compare(e, o, what):
    H.assert_same_state(e.store_state(), o.store_state(), what)


def random_raft_state(rng, G, R, K, max_term=6, max_log=12):
    """Random RAFT-mode state: votedFor+1 in 0..R, high-water marks at or
    above last (truncated logs) but inside the ring window, NextIndex rows."""
    st = H.random_state(rng, G, R, K, max_term, max_log)
    st["voted"][:] = rng.integers(0, R + 1, (G, R))
    for g in range(G):
        for r in range(R):
            last = int(st["last"][g, r])
            st["hwm"][g, r] = last + int(rng.integers(0, K)) if last > 0 else int(rng.integers(0, 3))
            # entries above last but inside the window are stale ring content
            for i in range(max(1, int(st["hwm"][g, r]) - K + 1), int(st["hwm"][g, r]) + 1):
                if i > last:
                    st["log_term"][g, r, (i - 1) % K] = rng.integers(0, max_term)
                    st["log_value"][g, r, (i - 1) % K] = rng.integers(0, 1 << 62)
            if st["role"][g, r] == abi.LEADER:
                for p in range(R):
                    if p != r:
                        st["next"][g, r, p] = rng.integers(0, last + 3)
    return st


@pytest.mark.parametrize("R,crc", [(1, 0), (2, 0), (3, 0), (4, 0), (5, 0), (7, 0), (8, 0), (3, 1), (5, 1)])
def test_raft_handler_batches_random_states(R, crc):
    rng = np.random.default_rng(7000 + R + 50 * crc)
    G, K = 192, 8
    e, o = pair(replicas=R, groups=G, ring_depth=K, seed=0xA11 + R, payload_crc=crc)
    st = random_raft_state(rng, G, R, K)
    if crc:
        H.stamp_crcs(st)
    e.load_state(st)
    o.load_state(st)
    compare(e, o, "after load")
    for rnd in range(15):
        now = int(rng.integers(0, 40))
        kind = rnd % 3
        groups = rng.permutation(G)[: G // 2]
        if kind == 0:
            items = []
            for g in groups:
                n = int(rng.integers(0, 12))
                items.append(dict(group=int(g), to=int(rng.integers(0, R)), term=int(rng.integers(0, 7)),
                                  prev_log_index=int(rng.integers(0, 14)), prev_log_term=int(rng.integers(0, 7)),
                                  leader_commit=int(rng.integers(0, 16)),
                                  logs=[(int(rng.integers(0, 7)), int(rng.integers(0, 1 << 62))) for _ in range(n)]))
            reqs, ents = H.ae_reqs(items)
            a, b = e.append_entries(now, reqs, ents), o.append_entries(now, reqs, ents)
        elif kind == 1:
            reqs = H.vote_reqs([dict(group=int(g), to=int(rng.integers(0, R)), term=int(rng.integers(0, 8)),
                                     candidate_id=int(rng.integers(0, R))) for g in groups])
            reqs["last_log_index"] = rng.integers(0, 14, len(reqs))
            reqs["last_log_term"] = rng.integers(0, 7, len(reqs))
            a, b = e.request_vote(now, reqs), o.request_vote(now, reqs)
        else:
            ops = H.ops([dict(group=int(g), replica=int(rng.integers(0, R)), kind=int(rng.integers(1, 6)),
                              arg=int(rng.integers(0, 1 << 62))) for g in groups])
            a, b = e.group_ops(now, ops), o.group_ops(now, ops)
        assert a.tobytes() == b.tobytes(), f"round {rnd} kind {kind}: responses differ"
        compare(e, o, f"round {rnd} kind {kind}")


@pytest.mark.parametrize("R", [3, 5])
def test_raft_random_state_ticks(R):
    rng = np.random.default_rng(9100 + R)
    G, K = 300, 16
    e, o = pair(replicas=R, groups=G, ring_depth=K, seed=0x7E + R, client_period=1,
                isolate_per_65536=12000, isolate_min_ticks=2, isolate_max_ticks=16)
    st = random_raft_state(rng, G, R, K)
    e.load_state(st)
    o.load_state(st)
    for t in range(30, 90, 3):
        a, b = e.tick(t, 3), o.tick(t, 3)
        assert list(a) == list(b), f"stats differ at tick {t}"
        compare(e, o, f"after tick {t + 2}")


TRACES = {
    # name: (config kwargs, init, first tick, ticks, compare every)
    "raft_newnode_r3": (dict(replicas=3, groups=512, client_period=5, seed=0x5EED0001), "new", 0, 200, 8),
    "raft_newnode_r5_iso": (dict(replicas=5, groups=384, client_period=1, seed=0x5EED0004, ring_depth=64,
                                 isolate_per_65536=16384, isolate_min_ticks=2, isolate_max_ticks=32),
                            "new", 0, 300, 10),
    "raft_newnode_r7_churn": (dict(replicas=7, groups=256, client_period=1, entries_per_tick=2, seed=0x44,
                                   ring_depth=64, isolate_per_65536=40000, isolate_min_ticks=1,
                                   isolate_max_ticks=32), "new", 0, 300, 10),
    "raft_steady_r5_iso": (dict(replicas=5, groups=512, client_period=1, ring_depth=32, seed=0x5EED0005,
                                isolate_per_65536=20000, isolate_min_ticks=4, isolate_max_ticks=20),
                           "steady0", 1, 200, 5),
    "raft_evict_small_ring": (dict(replicas=3, groups=300, client_period=1, entries_per_tick=3, ring_depth=8,
                                   seed=0xE1, isolate_per_65536=30000, isolate_min_ticks=4,
                                   isolate_max_ticks=24), "steady-1", 1, 150, 5),
    "raft_crc_corrupt": (dict(replicas=5, groups=200, client_period=1, entries_per_tick=8, ring_depth=64,
                              payload_crc=1, corrupt_per_65536=4000, isolate_per_65536=8000, seed=0xC5),
                         "new", 0, 120, 4),
    # bench.py's C4 workload parameters (R=7, K=64, 8-32 tick isolations at 1/8 per epoch) on 2048 groups
    "raft_c4_shape": (dict(replicas=7, groups=2048, client_period=1, seed=0x5EED0002, ring_depth=64,
                           isolate_per_65536=8192, isolate_min_ticks=8, isolate_max_ticks=32),
                      "new", 0, 400, 25),
    # SURVEY §8(d) C4 as specified: leader isolation (isolate_leader), at 2048 groups
    "raft_c4_leader_iso": (dict(replicas=7, groups=2048, client_period=1, seed=0x5EED0004, ring_depth=64,
                                isolate_per_65536=8192, isolate_min_ticks=8, isolate_max_ticks=32,
                                isolate_leader=1), "new", 0, 400, 25),
    "raft_leader_iso_r5_dense": (dict(replicas=5, groups=600, client_period=1, seed=0x1EAD, ring_depth=64,
                                      isolate_per_65536=40000, isolate_min_ticks=4, isolate_max_ticks=32,
                                      isolate_leader=1), "new", 0, 300, 10),
    "raft_r1": (dict(replicas=1, groups=64, client_period=1, seed=1), "new", 0, 60, 5),
    "raft_r2": (dict(replicas=2, groups=64, client_period=1, seed=2, isolate_per_65536=9000), "new", 0, 80, 5),
    "raft_r4": (dict(replicas=4, groups=300, client_period=1, seed=4, isolate_per_65536=9000), "new", 0, 120, 5),
    "raft_r8": (dict(replicas=8, groups=300, client_period=1, seed=8, isolate_per_65536=9000), "new", 0, 150, 5),
}


@pytest.mark.parametrize("name", sorted(TRACES))
def test_raft_tick_trace(name):
    kw, init, t0, n, every = TRACES[name]
    e, o = pair(**kw)
    for x in (e, o):
        if init == "new":
            x.init_new_nodes(t0)
        else:
            x.init_steady(-1 if init == "steady-1" else 0, t0 - 1 if t0 else 0)
    compare(e, o, "init")
    t = t0
    while t < t0 + n:
        k = min(every, t0 + n - t)
        a, b = e.tick(t, k), o.tick(t, k)
        assert list(a) == list(b), f"{name}: stats differ in ticks [{t}, {t + k})"
        ha = H.group_hashes(e.store_state(), raft_fields=True)
        hb = H.group_hashes(o.store_state(), raft_fields=True)
        bad = np.nonzero(ha != hb)[0]
        if bad.size:
            compare(e, o, f"{name}: after tick {t + k - 1} (groups {bad[:8].tolist()})")
        t += k
    compare(e, o, f"{name}: final")
    s = o.store_state()
    assert s["commit"].max() > 0, "trace made no progress"
