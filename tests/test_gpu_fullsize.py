"""GPU: every BASELINE config exactly as bench.py runs it, at full size,
against the CPU oracle — and proof that every fast-path class of the tick is
exercised by an oracle-compared run.

The workloads are taken from bench.WORKLOADS / bench.engine_kwargs (not
restated here), and the engine is driven with the bench's call structure
(settle, warm-up, then timed calls of 20 ticks). A whole 2^22-group oracle
would need ~100 GB of Go-slice logs, so the oracle runs SLICES: oracle
engines of SLICE groups started at global offsets (group_base) spread over
the engine, the first and the last groups included. Raft groups never
address each other (main.go:12, 259, 334) and the trace RNG is keyed by the
global group id, so a slice evolves exactly like those groups inside the big
engine. Compared: per-group digests of every slice after every call, and the
whole canonical state of every slice (raft_store_state_range vs the oracle's
view) at three points.

Class coverage: with raft_diag_enable the lean and list kernels count the
lanes that took each class of tick (include/raftstep.h raft_diag_counter).
The C4-config run on 2^16 groups is compared with ONE oracle over every
group (stats + digests per call, state at three points), so every class it
takes is oracle-checked; each must be taken >= 1000 times there.
"""
import numpy as np
import pytest

import bench
import harness as H
import oracle
from raftstep import Engine

pytestmark = pytest.mark.gpu
SLICE = 700
THREADS = 16
CALLS = [20] * 15    # the timed calls after settle + warm-up: 300 ticks, past the KP = 2K = 256-slot ring wrap


def workload_kwargs(name, groups=None):
    wl = bench.WORKLOADS[name]
    R = wl.get("replicas", bench.R_DEFAULT)
    G = groups or wl["groups"]
    return wl, bench.engine_kwargs(wl, R, G, 0, wl["ring_depth"], wl["entries"], wl["crc"])


def offsets(G, n=10, seed=7):
    rng = np.random.default_rng(seed)
    mid = sorted(int(x) for x in rng.integers(1, G - 2 * SLICE, n - 2))
    return [0] + mid + [G - SLICE]


def check_slices(e, slices, offs, what, full=False):
    d, _ = e.state_digest()
    for o, off in zip(slices, offs):
        do, _ = o.state_digest()
        bad = np.nonzero(d[off:off + SLICE] != do)[0]
        if bad.size:
            g = int(bad[0])
            raise AssertionError(f"{what}: slice at {off}: {bad.size} group digests differ, first local {g} "
                                 f"(group {off + g})\nengine:\n{e.nodelog(off + g)}oracle:\n{o.nodelog(g)}")
        if full:
            H.assert_same_state(e.store_state_range(off, SLICE), o.store_state(), f"{what}, slice at {off}")


def run_sliced(name, init, calls, groups=None, state_at=(0, 7, None)):
    """Runs workload `name` as bench.py does (init, then the calls), with
    oracle slices; returns the engine's class counters and the stats sum."""
    wl, kw = workload_kwargs(name, groups)
    G = kw["groups"]
    e = Engine(**kw)
    offs = offsets(G)
    slices = [oracle.Oracle(**dict(kw, groups=SLICE, group_base=off)) for off in offs]
    e.diag_enable()
    for x in [e] + slices:
        if init == "new":
            x.init_new_nodes(0)
        else:
            x.init_steady(0, 0)
    t = 0 if init == "new" else 1
    total = np.zeros(8, np.int64)
    points = {len(calls) - 1 if p is None else p for p in state_at}
    for i, k in enumerate(calls):
        total += e.tick(t, k)
        for o in slices:
            o.tick(t, k, threads=THREADS)
        t += k
        check_slices(e, slices, offs, f"{name} after tick {t - 1}", full=i in points)
    cls = e.diag_read()
    e.close()
    for o in slices:
        o.close()
    return cls, total, t


def test_c4_as_benchmarked_full_size():
    """bench.py --workload C4 verbatim: 2^22 groups, R=7, K=128 (KP=256),
    NewNode start, leader isolation (isolate_leader=1), seed 0x5EED0004, RAFT
    semantics; 48 settle ticks, 5 warm-up, then 300 ticks past the ring wrap.
    Anchors: elections main.go:171-177 / 253-284, step-down 309-320, the
    follower AppendEntries handler 135-149 (RAFT: truncate on conflict)."""
    wl = bench.WORKLOADS["C4"]
    assert wl["iso"][3] == 1 and wl["semantics"] == 1 and wl["seed"] == 0x5EED0004 and wl["groups"] == 1 << 22
    cls, total, t = run_sliced("C4", "new", [wl["settle"], 5] + CALLS, state_at=(0, 8, None))
    assert t == wl["settle"] + 5 + 300
    assert total[6] == 0, "no group may fault in RAFT mode"
    # the churn really happened at full size (every class of the C4 tick)
    for k in ("list_election", "list_first_round", "list_return", "list_stale", "lean_lxs", "list_window_start",
              "lean_sxs", "list_sxs_entered"):
        assert cls[k] > 10000, (k, cls)


def test_c4ref_as_benchmarked_full_size():
    """bench.py --workload C4REF verbatim (REF semantics, main.go bit for bit):
    groups freeze on their first fault — KAT-11's panic at a new leader's
    first contact (main.go:142 -> 404) — and every fault code must match the
    oracle group for group (the digest covers the fault code)."""
    wl = bench.WORKLOADS["C4REF"]
    assert wl["semantics"] == 0 and wl["iso"][3] == 1
    cls, total, t = run_sliced("C4REF", "new", [wl["settle"], 5] + CALLS[:6], state_at=(0, 4, None))
    assert total[6] > 0, "REF must fault under leader churn (KAT-11)"


def test_c5_as_benchmarked_full_size():
    """bench.py --workload C5 verbatim: 2^20 groups, E=64 entries per tick,
    K=128, CRC32C stamp + verify (EXT), seed 0x5EED0005; 48 ticks (the ring
    wraps every 2 ticks)."""
    wl = bench.WORKLOADS["C5"]
    assert wl["entries"] == 64 and wl["crc"] == 1
    cls, total, t = run_sliced("C5", "steady", [5, 20, 20, 3], state_at=(0, 2, None))
    assert total[0] == (1 << 20) * 64 * (t - 1) and total[6] == 0   # every tick commits its E entries


def test_c2_as_benchmarked_full_size_slices():
    """bench.py default (C2) verbatim through the bench's call structure,
    whole canonical state of the slices (the digest test covers every group)."""
    cls, total, t = run_sliced("C2", "steady", [5, 20, 20, 20], state_at=(0, 2, None))
    assert total[6] == 0
    assert cls["ticks_list_skipped"] >= 40, cls   # the steady-state list skip ran, and stayed exact


MIN_TAKEN = 1000


@pytest.mark.parametrize("vx", ["1", "0"], ids=["virtual_suffix", "stored_suffix"])
def test_class_coverage_c4_config_full_oracle(monkeypatch, vx):
    """C4's configuration (R=7, K=128, leader isolation, RAFT, seed
    0x5EED0004) on 2^16 groups against ONE oracle over every group — stats
    and per-group digests after every call, the whole canonical state at
    three points — with the tick-class counters on: every fast-path class of
    the lean and list kernels is taken >= 1000 times in this oracle-compared
    run (elections, first rounds, stale leaders, returns with truncation,
    LXS, HWX, three-segment switches, window starts, quiet leaderless ticks).
    With virtual suffixes (M_VX, the default) the cut-off leaders' entries are
    regenerated, their returns copy nothing and no switch moves them (the
    digests after every call materialise the suffixes, so both forms run);
    RAFTSTEP_VX=0 stores them, copies them back and moves them."""
    monkeypatch.setenv("RAFTSTEP_VX", vx)
    _, kw = workload_kwargs("C4", groups=1 << 16)
    e = Engine(**kw)
    o = oracle.Oracle(**kw)
    e.diag_enable()
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    calls = [48, 5] + [20] * 20   # 453 ticks
    for i, k in enumerate(calls):
        se = e.tick(t, k)
        so = o.tick(t, k, threads=THREADS)
        assert list(se) == list(so), f"stats [{t}, {t + k})"
        t += k
        de, te = e.state_digest()
        do, to = o.state_digest()
        bad = np.nonzero(de != do)[0]
        assert not bad.size, f"after tick {t - 1}: {bad.size} digests differ, first {bad[:8].tolist()}"
        assert te == to
        if i in (0, 10, len(calls) - 1):
            H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
    cls = e.diag_read()
    print("class counters:", cls)
    need = ["lean_ssync", "lean_lxs", "lean_lxs_whole_row", "lean_switch", "lean_three_seg", "lean_hwx",
            "list_quiet", "list_isolated_leader", "list_election", "list_first_round", "list_return",
            "list_return_trunc", "list_stale", "list_hwx", "list_window_start", "list_switch", "lean_sxs",
            "list_sxs_entered", "list_sxs_materialised"]
    need += ["lean_sxs_vx", "list_return_vx", "list_lxs_vx"] if vx == "1" else \
        ["lean_sxs_stale_in_row", "list_stale_moved"]
    low = {k: cls[k] for k in need if cls[k] < MIN_TAKEN}
    assert not low, f"classes taken fewer than {MIN_TAKEN} times: {low}\nall: {cls}"


def test_class_coverage_isolated_replica_and_three_segments():
    """The classes leader isolation does not reach: an isolated follower
    (hashed-victim windows, round 1's C4R) whose election timer fires while
    cut off, and ring segment switches in the list kernel — C4R's
    configuration on 2^15 groups against one oracle over every group."""
    _, kw = workload_kwargs("C4R", groups=1 << 15)
    e = Engine(**kw)
    o = oracle.Oracle(**kw)
    e.diag_enable()
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    for k in [48, 5] + [20] * 20:
        assert list(e.tick(t, k)) == list(o.tick(t, k, threads=THREADS)), f"stats [{t}, {t + k})"
        t += k
        assert e.state_digest()[1] == o.state_digest()[1], f"digest after tick {t - 1}"
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
    cls = e.diag_read()
    print("class counters:", cls)
    need = ["list_isolated_replica", "list_timer_fire", "list_quiet", "lean_ssync"]
    low = {k: cls[k] for k in need if cls[k] < MIN_TAKEN}
    assert not low, f"classes taken fewer than {MIN_TAKEN} times: {low}\nall: {cls}"
