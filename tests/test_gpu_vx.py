"""GPU: virtual log suffixes (raft_device.hpp M_VX, round 5). Under C4's
leader isolation a cut-off leader's own entries are regenerated from the
trace RNG instead of stored, its ring column mirrors the new primary's
entries, and its return needs no copy; every other reader materialises the
suffix first (the general kernel at load, the engine before host reads and
handler batches, and before a call that does not start at the tick after the
last one). These tests keep suffixes alive ACROSS calls (no host read in
between, unlike the digest-per-call tests) and then check the whole state
against the oracle, and exercise each materialisation trigger.
Anchors: main.go:171-177 (timeouts), 253-284 (elections), 309-320 (step-down),
327-329 (client append), 121-156 (AppendEntries)."""
import numpy as np
import pytest

import bench
import harness as H
import oracle
from raftstep import Engine

pytestmark = pytest.mark.gpu


def _kw(groups=1 << 13, churn=4):
    wl = bench.WORKLOADS["C4"]
    kw = bench.engine_kwargs(wl, 7, groups, 0, wl["ring_depth"], 1, 0)
    kw["isolate_per_65536"] = churn * wl["iso"][0]
    return kw


def _check(e, o, what):
    de, te = e.state_digest()
    do, to = o.state_digest()
    bad = np.nonzero(de != do)[0]
    assert not bad.size, f"{what}: {bad.size} digests differ, first group {int(bad[0])}\n" \
                         f"engine:\n{e.nodelog(int(bad[0]))}oracle:\n{o.nodelog(int(bad[0]))}"
    assert te == to
    H.assert_same_state(e.store_state(), o.store_state(), what)


@pytest.mark.parametrize("calls", [[48] + [20] * 12, [48, 1, 2, 3, 5, 8, 13, 21, 34, 55]])
def test_virtual_suffixes_across_calls(calls):
    """Calls back to back with statistics only (no host read of the state):
    suffixes live across call boundaries; the stats of every call, then the
    digests and the whole canonical state at the end, equal the oracle's."""
    kw = _kw()
    e, o = Engine(**kw), oracle.Oracle(**kw)
    e.diag_enable()
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    for k in calls:
        assert list(e.tick(t, k)) == list(o.tick(t, k, threads=16)), f"stats of ticks [{t}, {t + k})"
        t += k
    cls = e.diag_read()
    assert cls["list_lxs_vx"] > 100 and cls["list_return_vx"] > 100 and cls["lean_sxs_vx"] > 100, cls
    _check(e, o, f"after tick {t - 1}")


def test_virtual_suffixes_flushed_by_a_tick_gap_and_host_reads():
    """The triggers: a call that starts later than the tick after the last
    one (the suffixes are defined by consecutive client ticks), a host read of
    a group's words and of a state range in between calls, and stats-less
    calls."""
    kw = _kw()
    e, o = Engine(**kw), oracle.Oracle(**kw)
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    e.tick(0, 48)
    o.tick(0, 48, threads=16)
    e.tick(48, 20, stats=False)
    o.tick(48, 20, threads=16)
    # a gap of 9 ticks (nothing runs in them, as for the oracle)
    assert list(e.tick(77, 20)) == list(o.tick(77, 20, threads=16))
    e.debug_group_words(17)                       # host read: flush
    assert list(e.tick(97, 15)) == list(o.tick(97, 15, threads=16))
    ow = o.store_state()
    H.assert_same_state(e.store_state_range(100, 700), {k: v[100:800] for k, v in ow.items()}, "range after tick 111")
    assert list(e.tick(112, 30)) == list(o.tick(112, 30, threads=16))
    _check(e, o, "after tick 141")


def test_stored_suffixes_knob_matches():
    """RAFTSTEP_VX=0 (stored suffixes, copies and moves) over the same calls."""
    import os
    os.environ["RAFTSTEP_VX"] = "0"
    try:
        kw = _kw()
        e = Engine(**kw)
    finally:
        del os.environ["RAFTSTEP_VX"]
    o = oracle.Oracle(**kw)
    e.diag_enable()
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    for k in [48] + [20] * 6:
        assert list(e.tick(t, k)) == list(o.tick(t, k, threads=16))
        t += k
    cls = e.diag_read()
    assert cls["list_lxs_vx"] == 0 and cls["list_return_vx"] == 0 and cls["list_stale_moved"] > 0, cls
    _check(e, o, f"after tick {t - 1}")
