"""GPU: the engine's own run-time checks and audit surface added for the
steady-state list skip (engine.cpp): a group the lean kernel passes on while
the list kernel is skipped must fail loudly — in the call with statistics
itself, and in the call after a stats-less one — and poison the engine until
its state is replaced; the check zeroes the list counters (no stale list
entries for a later list kernel); raft_tick_records refuses more records than
the last call produced; raft_store_state_range equals the slice of the whole
view."""
import numpy as np
import pytest

import harness as H
import oracle
from raftstep import Engine, RaftError, abi

pytestmark = pytest.mark.gpu
KW = dict(replicas=5, groups=3000, ring_depth=16, client_period=1, seed=0x5EED0002)


@pytest.fixture(params=[1, 16], ids=["one_tick_per_launch", "fused16"])
def tpl(request):
    """raft_config.ticks_per_launch: the §8(d) form and the fused steady ticks"""
    return request.param


def steady_pair(tpl=1):
    e, o = Engine(ticks_per_launch=tpl, **KW), oracle.Oracle(**KW)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    assert list(e.tick(1, 6)) == list(o.tick(1, 6))   # proves the list empty: the next calls skip it
    e.diag_enable()
    return e, o


def test_forced_pass_is_exact_while_the_list_kernel_runs():
    e, o = Engine(**KW), oracle.Oracle(**KW)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    e.debug_force_pass(17)
    e.diag_enable()
    for t, k in ((1, 6), (7, 9)):   # the first call proves nothing (group 17 is always listed): no skip
        assert list(e.tick(t, k)) == list(o.tick(t, k))
    H.assert_same_state(e.store_state(), o.store_state(), "forced pass, list kernel running")
    c = e.diag_read()
    # every tick the lean kernel either passes group 17 on or (pipelined tick)
    # leaves it to the list kernel that carries it through that tick (so at
    # least every other tick, and every tick without the pipeline); the
    # skipped lanes also hold every group of the first tick after
    # init_steady, which the list kernel compresses and carries
    assert c["lean_forced"] >= 8 and c["lean_forced"] + c["lean_skipped"] >= 15, c
    assert c["ticks_list_skipped"] == 0, c


def test_skip_violation_fails_in_the_call_with_statistics(tpl):
    e, o = steady_pair(tpl)
    assert list(e.tick(7, 5)) == list(o.tick(7, 5))    # skipped and exact
    assert e.diag_read()["ticks_list_skipped"] == 5
    e.debug_force_pass(42)
    with pytest.raises(RaftError, match="list kernel that did not run") as ei:
        e.tick(12, 4)
    assert ei.value.code == abi.RAFT_EINTERNAL
    # poisoned: every call fails until the state is replaced
    for call in (lambda: e.tick(16, 1), e.store_state, e.state_digest, e.sync):
        with pytest.raises(RaftError, match="engine state is invalid"):
            call()
    e.debug_force_pass(-1)
    e.load_state(o.store_state())
    o.tick(12, 4)
    e.tick(12, 4)   # (first call after a load: the list kernel runs, nothing stale is on the list)
    H.assert_same_state(e.store_state(), o.store_state(), "after reload")


def test_skip_violation_fails_at_the_call_after_a_stats_less_call(tpl):
    e, o = steady_pair(tpl)
    e.tick(7, 5, stats=False)             # skipped, checked at the next call: clean
    e.tick(12, 3, stats=False)
    e.debug_force_pass(99)
    e.tick(15, 3, stats=False)            # the violation happens here (asynchronously)
    with pytest.raises(RaftError, match="ticks lost") as ei:
        e.tick(18, 1, stats=False)        # ... and is reported by the next call
    assert ei.value.code == abi.RAFT_EINTERNAL
    with pytest.raises(RaftError, match="engine state is invalid"):
        e.sync()
    e.init_steady(0, 0)                   # state replaced: usable again
    e.debug_force_pass(-1)
    o2 = oracle.Oracle(**KW)
    o2.init_steady(0, 0)
    assert list(e.tick(1, 6)) == list(o2.tick(1, 6))
    H.assert_same_state(e.store_state(), o2.store_state(), "after init_steady")


def test_stats_less_skipped_calls_stay_exact(tpl):
    e, o = steady_pair(tpl)
    t = 7
    for k in (5, 1, 13, 2):
        e.tick(t, k, stats=False)
        o.tick(t, k)
        t += k
    e.sync()
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
    c = e.diag_read()
    assert c["ticks_list_skipped"] == 21 and c["general_launches"] == 0, c
    assert list(e.tick(t, 4)) == list(o.tick(t, 4))


def test_failed_state_replacement_keeps_the_poison(tmp_path, tpl):
    """a call that would replace the state but fails before doing
    so (missing checkpoint, bad view, out-of-range tick) leaves a poisoned
    engine poisoned; a successful replacement clears it."""
    e, o = steady_pair(tpl)
    assert list(e.tick(7, 5)) == list(o.tick(7, 5))
    e.debug_force_pass(42)
    with pytest.raises(RaftError, match="list kernel that did not run"):
        e.tick(12, 4)
    e.debug_force_pass(-1)
    with pytest.raises(RaftError):
        e.load_checkpoint(tmp_path / "missing.ckpt")
    with pytest.raises(RaftError):
        e.init_steady(0, 1 << 40)         # virtual time out of int32: refused before any launch
    bad = o.store_state()
    bad["role"] = np.full_like(bad["role"], 9)
    with pytest.raises(RaftError):
        e.load_state(bad)
    with pytest.raises(RaftError, match="engine state is invalid") as ei:
        e.tick(12, 1)
    assert ei.value.code == abi.RAFT_EINTERNAL
    e.load_state(o.store_state())         # replaced: usable again
    assert list(e.tick(12, 3)) == list(o.tick(12, 3))
    H.assert_same_state(e.store_state(), o.store_state(), "after the reload")


def test_tick_records_refuses_more_than_the_last_call_produced():
    e = Engine(**KW)
    e.init_steady(0, 0)
    with pytest.raises(RaftError) as ei:
        e.tick_records(1)                 # no call with statistics yet
    assert ei.value.code == abi.RAFT_ERANGE
    e.tick(1, 10)
    e.tick(11, 3)
    assert e.tick_records(3).shape == (3, 8)
    with pytest.raises(RaftError) as ei:
        e.tick_records(4)                 # the previous call's records are gone
    assert ei.value.code == abi.RAFT_ERANGE


@pytest.mark.parametrize("sem", [abi.SEM_REF, abi.SEM_RAFT])
def test_store_state_range_is_the_slice_of_the_whole_view(sem):
    kw = dict(replicas=7, groups=1000, ring_depth=16, client_period=1, seed=0x77, semantics=sem,
              isolate_per_65536=20000, isolate_leader=1, payload_crc=1)
    e = Engine(**kw)
    e.init_new_nodes(0)
    e.tick(0, 120)
    whole = e.store_state()
    for g0, n in ((0, 1000), (0, 1), (63, 2), (64, 64), (130, 333), (999, 1), (511, 489)):
        part = e.store_state_range(g0, n)
        sl = {k: v[g0:g0 + n] for k, v in whole.items()}
        H.assert_same_state(part, sl, f"range [{g0}, +{n})")
    for g0, n in ((0, 0), (1000, 1), (990, 11)):
        with pytest.raises(RaftError) as ei:
            e.store_state_range(g0, n)
        assert ei.value.code == abi.RAFT_ERANGE


def test_engine_loads_version_1_checkpoints(tmp_path):
    """a checkpoint written before leader isolation (version 1, no
    iso_victim field) still loads; the victims load as none."""
    from raftstep import checkpoint
    kw = dict(replicas=5, groups=300, ring_depth=16, client_period=1, seed=0xC0DE, isolate_per_65536=12000)
    a = Engine(**kw)
    a.init_new_nodes(0)
    a.tick(0, 50)
    st = a.store_state()
    p = tmp_path / "v1.bin"
    checkpoint.write(p, a.cfg, st, version=1)
    b = Engine(**kw)
    b.load_checkpoint(p)
    H.assert_same_state(b.store_state(), st, "v1 checkpoint")   # (hashed victims: iso_victim is 0 anyway)
    assert list(a.tick(50, 20)) == list(b.tick(50, 20))


@pytest.mark.parametrize("split", ["1", "0"])
def test_split_steady_tick_matches_oracle(monkeypatch, split):
    """The steady tick split over two streams (engine.cpp split_steady: two
    launches per tick over the two halves of the groups, joined before every
    statistics reduce) against the oracle: enough groups for the split
    (>= 2 x 65536), a count that leaves a partial last block, calls with and
    without statistics, with the list skipped from the second call on."""
    monkeypatch.setenv("RAFTSTEP_SPLIT_STEADY", split)
    kw = dict(replicas=5, groups=(1 << 17) + 300, ring_depth=16, client_period=1, seed=0x5EED0002)
    e, o = Engine(**kw), oracle.Oracle(**kw)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    e.diag_enable()
    t = 1
    for k, st in ((6, True), (20, True), (7, False), (1, True), (13, False), (9, True)):
        se = e.tick(t, k, stats=st)
        so = o.tick(t, k, threads=16)
        if st:
            assert list(se) == list(so), f"stats of ticks [{t}, {t + k})"
        t += k
    e.sync()
    assert e.state_digest()[1] == o.state_digest()[1]
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
    c = e.diag_read()
    assert c["ticks_list_skipped"] >= 40, c


def test_debug_diag_mode_needs_the_wrong_results_flag():
    """raft_debug_diag_mode (timing diagnostics, results wrong) is refused
    unless the engine was created with RAFT_DEBUG_ALLOW_WRONG_RESULTS; mode 0
    (exact) is always accepted."""
    e = Engine(**KW)
    with pytest.raises(RaftError) as ei:
        e.debug_diag_mode(512)
    assert ei.value.code == -22
    e.debug_diag_mode(0)
    d = Engine(debug_flags=abi.DEBUG_ALLOW_WRONG_RESULTS, **KW)
    d.debug_diag_mode(512)
    d.debug_diag_mode(0)


def test_stream_probe_reports_its_bytes():
    """raft_stream_probe: the lean kernel's byte mix on fresh buffers (bench.py
    prices the lean kernel against it): 40 + 12 R bytes per element."""
    from raftstep import stream_probe
    us, by = stream_probe(0, 5, 1 << 20, 3)
    assert by == (1 << 20) * 100 and 0 < us < 1e5
    us7, by7 = stream_probe(0, 7, 1000, 2)
    assert by7 == 1024 * 124 and us7 > 0
    us1, by1 = stream_probe(0, 1, 1 << 20, 3, heartbeat=False)   # (the shared-form mix: 36 + 12 B)
    assert by1 == (1 << 20) * 48 and 0 < us1 < 1e5
    # the mode is an explicit argument, not the process environment
    us2, by2 = stream_probe(0, 1, 1 << 20, 3, flags=abi.PROBE_NO_HEARTBEAT | abi.PROBE_NT_RECORD)
    assert by2 == by1 and 0 < us2 < 1e5
    with pytest.raises(RaftError):
        stream_probe(0, 9, 1 << 20, 1)
    with pytest.raises(RaftError):
        stream_probe(0, 5, 1 << 20, 1, flags=8)
