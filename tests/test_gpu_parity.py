"""Differential parity: HIP engine vs the CPU oracle on identical seeded
inputs — handler batches on random states, and whole tick traces compared
field by field every few ticks. Bit-exact (integer state, no tolerance)."""
import numpy as np
import pytest

import harness as H
from raftstep import Engine, abi

pytestmark = pytest.mark.gpu


def pair(general=False, single=False, **kw):
    """(engine, oracle) on the same config. general=True routes every group
    through the general tick kernel (debug knob RAFTSTEP_FORCE_GENERAL);
    single=True runs the one-pass steady-state kernel instead of the default
    two-pass plan (lean kernel + list kernel, RAFTSTEP_TWO_PASS=0), so every
    device path is checked against the oracle on the same traces."""
    import os

    import oracle
    env = {"RAFTSTEP_FORCE_GENERAL": "1" if general else "0", "RAFTSTEP_TWO_PASS": "0" if single else "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e = Engine(**kw)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    return e, oracle.Oracle(**kw)


def compare(e, o, what):
    H.assert_same_state(e.store_state(), o.store_state(), what)


@pytest.mark.parametrize("R,crc", [(1, 0), (2, 0), (3, 0), (4, 0), (5, 0), (6, 0), (7, 0), (8, 0), (3, 1), (5, 1)])
def test_handler_batches_random_states(R, crc):
    rng = np.random.default_rng(1000 + R + 50 * crc)
    G, K = 192, 8
    e, o = pair(replicas=R, groups=G, ring_depth=K, seed=0xABC + R, payload_crc=crc)
    st = H.random_state(rng, G, R, K)
    if crc:
        H.stamp_crcs(st)
    e.load_state(st)
    o.load_state(st)
    compare(e, o, "after load")
    for rnd in range(12):
        now = int(rng.integers(0, 40))
        kind = rnd % 3
        groups = rng.permutation(G)[: G // 2]
        if kind == 0:
            items = []
            for g in groups:
                n = int(rng.integers(0, 12))
                items.append(dict(group=int(g), to=int(rng.integers(0, R)), term=int(rng.integers(0, 7)),
                                  prev_log_index=int(rng.integers(-1, 14)), prev_log_term=int(rng.integers(0, 7)),
                                  leader_commit=int(rng.integers(0, 16)),
                                  logs=[(int(rng.integers(0, 7)), int(rng.integers(0, 1 << 62))) for _ in range(n)]))
            reqs, ents = H.ae_reqs(items)
            a, b = e.append_entries(now, reqs, ents), o.append_entries(now, reqs, ents)
        elif kind == 1:
            reqs = H.vote_reqs([dict(group=int(g), to=int(rng.integers(0, R)), term=int(rng.integers(0, 8)))
                                for g in groups])
            a, b = e.request_vote(now, reqs), o.request_vote(now, reqs)
        else:
            ops = H.ops([dict(group=int(g), replica=int(rng.integers(0, R)), kind=int(rng.integers(1, 6)),
                              arg=int(rng.integers(0, 1 << 62))) for g in groups])
            a, b = e.group_ops(now, ops), o.group_ops(now, ops)
        assert a.tobytes() == b.tobytes(), f"round {rnd} kind {kind}: responses differ"
        compare(e, o, f"round {rnd} kind {kind}")


TRACES = {
    # name: (config kwargs, init, first tick, ticks, compare every)
    "newnode_r3": (dict(replicas=3, groups=512, client_period=5, seed=0x5EED0001), "new", 0, 240, 8),
    "newnode_r5_iso": (dict(replicas=5, groups=384, client_period=1, seed=0x5EED0004,
                            isolate_per_65536=16384, isolate_min_ticks=8, isolate_max_ticks=32), "new", 0, 300, 10),
    "newnode_r7_iso": (dict(replicas=7, groups=256, client_period=2, entries_per_tick=2, seed=0x5EED0044,
                            isolate_per_65536=30000, isolate_min_ticks=1, isolate_max_ticks=32), "new", 0, 300, 10),
    "steady_r5_hashed": (dict(replicas=5, groups=640, client_period=1, entries_per_tick=3, ring_depth=8,
                              seed=0x5EED0002), "steady-1", 1, 120, 6),
    "steady_r5_iso": (dict(replicas=5, groups=512, client_period=1, ring_depth=16, seed=0x5EED0005,
                           isolate_per_65536=20000, isolate_min_ticks=4, isolate_max_ticks=20), "steady0", 1, 200, 5),
    "wrap_e_gt_k": (dict(replicas=3, groups=130, client_period=3, entries_per_tick=40, ring_depth=16,
                         seed=0x77), "steady0", 1, 40, 1),
    "steady_e7_k8": (dict(replicas=5, groups=700, client_period=1, entries_per_tick=7, ring_depth=8,
                          seed=0x78), "steady-1", 1, 30, 3),
    "steady_heartbeats": (dict(replicas=3, groups=260, client_period=4, entries_per_tick=2, ring_depth=8,
                               seed=0x79), "steady0", 1, 40, 1),
    "c5_crc_corrupt": (dict(replicas=5, groups=200, client_period=1, entries_per_tick=64, ring_depth=128,
                            payload_crc=1, corrupt_per_65536=3000, seed=0x5EED0005), "steady0", 1, 16, 2),
    "crc_newnode_iso": (dict(replicas=3, groups=300, client_period=1, entries_per_tick=2, ring_depth=16,
                             payload_crc=1, corrupt_per_65536=5000, isolate_per_65536=12000,
                             seed=0xC5C), "new", 0, 150, 5),
    # EXT leader-isolation mode: the window's victim is the leader at its first tick
    "leader_iso_r3": (dict(replicas=3, groups=400, client_period=1, seed=0x5EED0014, isolate_per_65536=20000,
                           isolate_leader=1), "new", 0, 240, 8),
    "leader_iso_steady_r5": (dict(replicas=5, groups=500, client_period=1, ring_depth=16, seed=0x5EED0015,
                                  isolate_per_65536=30000, isolate_min_ticks=4, isolate_max_ticks=24,
                                  isolate_leader=1), "steady0", 1, 200, 5),
    "r1": (dict(replicas=1, groups=64, client_period=1, seed=1), "new", 0, 60, 5),
    "r2": (dict(replicas=2, groups=64, client_period=1, seed=2), "new", 0, 60, 5),
    "r4": (dict(replicas=4, groups=300, client_period=1, seed=4), "new", 0, 120, 5),
    "r6": (dict(replicas=6, groups=300, client_period=1, seed=6, isolate_per_65536=9000), "new", 0, 150, 5),
    "r8": (dict(replicas=8, groups=300, client_period=1, seed=8, isolate_per_65536=9000), "new", 0, 150, 5),
}


@pytest.mark.parametrize("path", ["auto", "single", "general"])
@pytest.mark.parametrize("name", sorted(TRACES))
def test_tick_trace(name, path):
    kw, init, t0, n, every = TRACES[name]
    e, o = pair(general=(path == "general"), single=(path == "single"), **kw)
    for x in (e, o):
        if init == "new":
            x.init_new_nodes(t0)
        else:
            x.init_steady(-1 if init == "steady-1" else 0, t0 - 1 if t0 else 0)
    compare(e, o, "init")
    t = t0
    tot_e = np.zeros(8, np.int64)
    tot_o = np.zeros(8, np.int64)
    while t < t0 + n:
        k = min(every, t0 + n - t)
        tot_e += e.tick(t, k)
        tot_o += o.tick(t, k)
        t += k
        compare(e, o, f"{name} after tick {t - 1}")
        assert list(tot_e) == list(tot_o), f"stats differ after tick {t - 1}: {tot_e} vs {tot_o}"


def test_tick_from_random_states():
    """Random (well-formed) states exercise multi-leader groups, stale
    candidates, deadlocks and panics inside the fused tick."""
    for R, crc in ((3, 0), (5, 0), (7, 0), (5, 1)):
        rng = np.random.default_rng(77 + R + crc)
        G, K = 512, 16
        kw = dict(replicas=R, groups=G, ring_depth=K, client_period=2, seed=900 + R, isolate_per_65536=8000,
                  payload_crc=crc, corrupt_per_65536=6000 * crc)
        e, o = pair(**kw)
        st = H.random_state(rng, G, R, K)
        if crc:
            H.stamp_crcs(st)
        e.load_state(st)
        o.load_state(st)
        for t in range(30, 60):
            se, so = e.tick(t, 1), o.tick(t, 1)
            assert list(se) == list(so), (R, t)
            compare(e, o, f"R={R} tick {t}")


def test_full_size_steady_state_properties():
    """BASELINE config C2 at full size (2^20 groups, R=5, E=1): size-independent
    properties of the steady state after N ticks (every log has N entries,
    leader commit N, followers N-1, per-tick stats in closed form), plus a
    bit-exact oracle diff of a slice of groups run through an oracle that
    owns just that slice (group_base)."""
    import oracle
    G, R, N = 1 << 20, 5, 24
    kw = dict(replicas=R, groups=G, ring_depth=32, client_period=1, entries_per_tick=1, seed=0x5EED0002)
    e = Engine(**kw)
    e.init_steady(0, 0)
    stats = e.tick(1, N)
    assert list(stats) == [G * N, 0, 0, 4 * G * N, 0, 0, 0, G * N]
    st = e.store_state(logs=False)
    assert (st["last"] == N).all() and (st["fault"] == 0).all()
    assert (st["commit"][:, 0] == N).all() and (st["commit"][:, 1:] == N - 1).all()
    assert (st["deadline"][:, 1:] == 2 * N + st["timeout"][:, 1:]).all()
    full = e.store_state(logs=True)
    for g0 in (0, G // 2 + 123, G - 700):
        kw2 = dict(kw, groups=700, group_base=g0)
        o = oracle.Oracle(**kw2)
        o.init_steady(0, 0)
        o.tick(1, N)
        ref = o.store_state()
        sl = {k: v[g0:g0 + 700] for k, v in full.items()}
        H.assert_same_state(sl, ref, f"slice at {g0}")


@pytest.mark.parametrize("sem", [abi.SEM_REF, abi.SEM_RAFT])
def test_handler_batches_on_compressed_steady_groups(sem):
    """Groups the steady-state kernel keeps in compressed form (SSYNC: the
    term / LastApplied / CommitIndex / last-entry-term rows of a group held as
    one 16-B record) go through every handler batch, a nodelog and further
    ticks; every reader must see the rows the record stands for."""
    R, G, K = 5, 320, 16
    e, o = pair(replicas=R, groups=G, ring_depth=K, client_period=1, seed=0x5515 + sem, semantics=sem)
    for x in (e, o):
        x.init_steady(0, 0)
    assert list(e.tick(1, 6)) == list(o.tick(1, 6))
    compare(e, o, "after 6 steady ticks")
    assert e.nodelog(7) == o.nodelog(7)
    rng = np.random.default_rng(0x55 + sem)
    for rnd in range(9):
        now = 7 + 2 * rnd   # the handler batches' tick, between the fused ticks (time is monotone)
        kind = rnd % 3
        groups = rng.permutation(G)[: G // 3]
        if kind == 0:
            items = [dict(group=int(g), to=int(rng.integers(1, R)), term=int(rng.integers(1, 4)),
                          prev_log_index=int(rng.integers(4, 9)), prev_log_term=int(rng.integers(1, 3)),
                          leader_commit=int(rng.integers(0, 9)),
                          logs=[(int(rng.integers(1, 4)), int(rng.integers(0, 1 << 62)))
                                for _ in range(int(rng.integers(0, 3)))]) for g in groups]
            reqs, ents = H.ae_reqs(items)
            a, b = e.append_entries(now, reqs, ents), o.append_entries(now, reqs, ents)
        elif kind == 1:
            reqs = H.vote_reqs([dict(group=int(g), to=int(rng.integers(0, R)), term=int(rng.integers(1, 4)))
                                for g in groups])
            a, b = e.request_vote(now, reqs), o.request_vote(now, reqs)
        else:
            ops = H.ops([dict(group=int(g), replica=int(rng.integers(0, R)), kind=int(rng.integers(1, 6)),
                              arg=int(rng.integers(0, 1 << 62))) for g in groups])
            a, b = e.group_ops(now, ops), o.group_ops(now, ops)
        assert a.tobytes() == b.tobytes(), f"round {rnd} kind {kind}: responses differ"
        compare(e, o, f"round {rnd} kind {kind}")
        # the untouched groups are still compressed: tick everything once more
        se, so = e.tick(8 + 2 * rnd, 1), o.tick(8 + 2 * rnd, 1)
        assert list(se) == list(so), f"round {rnd}: tick stats differ"
        compare(e, o, f"round {rnd} tick")


@pytest.mark.parametrize("sem", [abi.SEM_REF, abi.SEM_RAFT])
def test_steady_state_list_skip(sem):
    """The engine's steady-state list skip (engine.cpp): after init_steady a
    call with statistics proves the list empty, the following calls run the
    lean kernel alone; a host mutation (here load_state of a state where one
    follower's CommitIndex lags, so the group is not compressed) must bring
    the list kernel back. Every step against the oracle, the whole state."""
    kw = dict(replicas=5, groups=3000, ring_depth=16, client_period=1, seed=0x5EED0002, semantics=sem)
    e, o = pair(**kw)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    t = 1
    for k in (6, 10, 13):   # establishes the skip, then skipped calls (and a ring wrap at K=16)
        assert list(e.tick(t, k)) == list(o.tick(t, k)), f"stats at {t}"
        compare(e, o, f"after tick {t + k - 1}")
        t += k
    st = o.store_state()
    st["commit"][7, 2] -= 1   # group 7, follower 2: one entry behind on CommitIndex
    e.load_state(st)
    o.load_state(st)
    for k in (1, 5, 8):
        assert list(e.tick(t, k)) == list(o.tick(t, k)), f"stats at {t} after the mutation"
        compare(e, o, f"after tick {t + k - 1} (mutated)")
        t += k
