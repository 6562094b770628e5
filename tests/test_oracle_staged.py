"""CPU: the oracle's staged client values (raft_config.client_source =
RAFT_CLIENT_STAGED, raftstep.h raft_stage_values) — the drop-in LogReq path
where the caller, not the trace RNG, supplies every rand.Int() of main.go:92
(main.go:87-93 -> 327-329).

Pinned two ways: (1) staging exactly the values the trace RNG would give the
steady leader reproduces the trace-mode run bit for bit (same state, same
digests, same stats) — the staged path changes where a value comes from and
nothing else; (2) every entry a leader appends holds the staged value of the
tick and slot that appended it (Log.Value, main.go:48), on every replica that
accepted it (main.go:148-149)."""
import numpy as np
import pytest

import bench
import harness as H
import oracle
from raftstep import abi


def _kw(**over):
    kw = dict(replicas=5, groups=48, ring_depth=16, client_period=1, entries_per_tick=2, seed=0x5EED0002)
    kw.update(over)
    return kw


def trace_values(o, first_tick, nticks, E, G, leader=0):
    """The trace RNG's values of `leader` (oracle_client_value) in staged layout [t][e][g]."""
    v = np.zeros((nticks, E, G), np.int64)
    for t in range(nticks):
        for e in range(E):
            for g in range(G):
                v[t, e, g] = o.client_value(o.cfg.group_base + g, leader, first_tick + t, e)
    return v


@pytest.mark.parametrize("sem", [0, 1])
def test_staged_leader_trace_values_reproduce_trace_mode(sem):
    kw = _kw(semantics=sem, group_base=1000)
    tr = oracle.Oracle(**kw)
    st = oracle.Oracle(**kw, client_source=abi.CLIENT_STAGED)
    for o in (tr, st):
        o.init_steady(0, 0)
    E, G = kw["entries_per_tick"], kw["groups"]
    t = 1
    for n in (3, 7, 10):
        st.stage_values(t, trace_values(tr, t, n, E, G, leader=0))
        a = tr.tick(t, n)
        b = st.tick(t, n)
        assert list(a) == list(b), (t, a, b)
        t += n
        assert (tr.state_digest()[0] == st.state_digest()[0]).all()
    H.assert_same_state(tr.store_state(), st.store_state(), "staged == trace")


def test_staged_values_land_in_every_accepting_log():
    kw = _kw(client_source=abi.CLIENT_STAGED, ring_depth=64)
    o = oracle.Oracle(**kw)
    o.init_steady(0, 0)
    E, G, R = kw["entries_per_tick"], kw["groups"], kw["replicas"]
    vals = bench.staged_values(kw["seed"], 0, G, 1, 12, E)
    o.stage_values(1, vals)
    o.tick(1, 12)
    st = o.store_state()
    for g in range(G):
        for r in range(R):
            log = H.log_of(st, g, r, kw["ring_depth"])
            assert len(log) == 12 * E
            # entry i (1-based) was appended at tick 1 + (i-1)//E, slot (i-1)%E
            assert [v for _, v in log] == [int(vals[i // E, i % E, g]) for i in range(12 * E)], (g, r)


def test_staged_ticks_outside_the_staged_range_are_refused():
    o = oracle.Oracle(**_kw(client_source=abi.CLIENT_STAGED))
    o.init_steady(0, 0)
    with pytest.raises(oracle.OracleError):
        o.tick(1, 2)                       # nothing staged yet
    o.stage_values(1, np.zeros((4, 2, 48), np.int64))
    o.tick(1, 4)
    with pytest.raises(oracle.OracleError):
        o.tick(5, 1)                       # past the staged range
    tr = oracle.Oracle(**_kw())
    with pytest.raises(oracle.OracleError):
        tr.stage_values(0, np.zeros((1, 2, 48), np.int64))   # trace-mode oracle: no staging


def test_bench_staged_values_are_sliceable():
    """An oracle slice (group_base offset) re-stages exactly its columns of the
    line's values (bench.staged_values is keyed by the global group id)."""
    a = bench.staged_values(0x5EED0004, 0, 5000, 48, 20, 3)
    b = bench.staged_values(0x5EED0004, 1234, 700, 50, 5, 3)
    assert (a[2:7, :, 1234:1934] == b).all()
    assert a.min() >= 0 and len(np.unique(a)) == a.size


def test_engine_rejects_unknown_client_source():
    """Config validation (before any HIP call)."""
    import ctypes as C
    from raftstep import engine
    lib = engine.load_library()
    c = abi.default_config(client_source=2)
    h = C.c_void_p()
    assert lib.raft_engine_create(C.byref(c), C.byref(h)) == abi.RAFT_EINVAL
    assert "client_source" in lib.raft_last_error().decode()
