"""GPU: shared entries (raft_device.hpp ROT_SH, round 5). While an SSYNC group
is taken by the lean (or fused) kernel's normal class, every replica receives
the same entries, so they are stored once, in the shared ring, and the group is
marked; every other reader copies them back into the R replica columns first
(the list kernel when it stages a passed group, the one-pass and general
kernels when they load one, the engine before host views and handler batches),
and the digest reads the shared ring itself. These tests keep shared entries
alive across calls and then check digests and the whole state against the
oracle, and exercise each copy-back trigger.
Anchors: main.go:121-156 (AppendEntries: every follower appends the entries it
received), 327-329 (client append), 341-391 (replication and commit)."""
import numpy as np
import pytest

import harness as H
import oracle
from raftstep import Engine

pytestmark = pytest.mark.gpu


def _pair(monkeypatch, sh=1, tpl=1, **kw):
    monkeypatch.setenv("RAFTSTEP_SH", str(sh))
    cfg = dict(replicas=5, groups=3000, ring_depth=16, client_period=1, seed=0x5EED0002, semantics=0)
    cfg.update(kw)
    return Engine(ticks_per_launch=tpl, **cfg), oracle.Oracle(**cfg)


def _digests(e, o, what):
    de, te = e.state_digest()
    do, to = o.state_digest()
    bad = np.nonzero(de != do)[0]
    assert not bad.size, f"{what}: {bad.size} digests differ, first group {int(bad[0])}\n" \
                         f"engine:\n{e.nodelog(int(bad[0]))}oracle:\n{o.nodelog(int(bad[0]))}"
    assert te == to


@pytest.mark.parametrize("R,crc,sem,E", [(3, 0, 0, 1), (5, 0, 1, 1), (7, 0, 1, 1), (5, 1, 0, 1), (5, 1, 1, 4),
                                         (4, 0, 0, 3)])
@pytest.mark.parametrize("tpl", [1, 16])
def test_shared_entries_across_calls(monkeypatch, R, crc, sem, E, tpl):
    """Calls back to back with statistics only: shared entries live across
    call boundaries and ring wraps (K=16); the digests (read from the shared
    ring, nothing copied back) and then the whole state (copied back by the
    host view) equal the oracle's, and ticking on after the copy-back stays
    exact."""
    e, o = _pair(monkeypatch, replicas=R, payload_crc=crc, semantics=sem, entries_per_tick=E, tpl=tpl)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    e.diag_enable()
    t = 1
    for k in (6, 10, 13, 1, 20):
        assert list(e.tick(t, k)) == list(o.tick(t, k)), f"stats of ticks [{t}, {t + k})"
        t += k
    cls = e.diag_read()
    if tpl == 1:
        assert cls["lean_sh"] > 3000 * 30, cls
    _digests(e, o, f"after tick {t - 1} (shared form)")
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
    assert list(e.tick(t, 9)) == list(o.tick(t, 9))
    t += 9
    _digests(e, o, f"after tick {t - 1}")
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")


def test_knob_off_gives_the_same_state(monkeypatch):
    """RAFTSTEP_SH=0 (every entry in the R replica columns) and the default
    reach the same digests tick for tick."""
    a, _ = _pair(monkeypatch, sh=1, replicas=5, payload_crc=1)
    b, _ = _pair(monkeypatch, sh=0, replicas=5, payload_crc=1)
    a.diag_enable()
    b.diag_enable()
    for x in (a, b):
        x.init_steady(0, 0)
    t = 1
    for k in (5, 17, 3):
        assert list(a.tick(t, k)) == list(b.tick(t, k))
        assert a.state_digest()[1] == b.state_digest()[1], f"after tick {t + k - 1}"
        t += k
    assert a.diag_read()["lean_sh"] > 0 and b.diag_read()["lean_sh"] == 0


def test_copy_back_by_the_list_kernel(monkeypatch):
    """A group in shared form the lean kernel passes on (the forced-pass test
    knob while the list kernel runs; a call after a tick gap, where every
    group is out of the global ring phase) is copied back by the list kernel
    when it stages it, and stays exact."""
    e, o = _pair(monkeypatch, replicas=5, semantics=1)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    e.diag_enable()
    e.tick(1, 20, stats=False)
    o.tick(1, 20)
    e.debug_force_pass(42)
    assert list(e.tick(21, 1)) == list(o.tick(21, 1))   # (a call with statistics: the list kernel runs)
    e.debug_force_pass(-1)
    assert e.diag_read()["list_sh_copied"] >= 1
    # a gap of 7 ticks (nothing runs in them, as for the oracle): every group
    # would drift out of the global phase, so the engine copies the shared
    # entries back before the call (the lean kernel then writes the drifted
    # groups' own segments, and takes them back into shared form once a ring
    # segment switch brings them into phase, where the ring has 2K slots)
    assert list(e.tick(29, 12)) == list(o.tick(29, 12))
    assert list(e.tick(41, 12)) == list(o.tick(41, 12))
    _digests(e, o, "after tick 52")
    H.assert_same_state(e.store_state(), o.store_state(), "after tick 52")


def test_copy_back_before_handler_batches_and_views(monkeypatch):
    """Host reads of a state range and a group's words, and a handler batch,
    each copy the shared entries back first; the ticks after them are exact."""
    e, o = _pair(monkeypatch, replicas=3, ring_depth=8)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    assert list(e.tick(1, 11)) == list(o.tick(1, 11))
    ow = o.store_state()
    H.assert_same_state(e.store_state_range(100, 700), {k: v[100:800] for k, v in ow.items()}, "range after tick 11")
    assert list(e.tick(12, 5)) == list(o.tick(12, 5))
    e.debug_group_words(17)
    assert list(e.tick(17, 5)) == list(o.tick(17, 5))
    # an AppendEntries batch straight after the ticks (no host read in
    # between): the handler path reads the rings (prevLogIndex / prevLogTerm
    # checks, conflicting suffixes) and writes them
    rng = np.random.default_rng(0x5A)
    items = [dict(group=int(g), to=int(rng.integers(1, 3)), term=int(rng.integers(1, 3)),
                  prev_log_index=int(rng.integers(14, 22)), prev_log_term=1, leader_commit=int(rng.integers(0, 22)),
                  logs=[(1, int(rng.integers(0, 1 << 62))) for _ in range(int(rng.integers(0, 3)))])
             for g in rng.permutation(3000)[:700]]
    reqs, ents = H.ae_reqs(items)
    a, b = e.append_entries(22, reqs, ents), o.append_entries(22, reqs, ents)
    assert a.tobytes() == b.tobytes(), "AppendEntries responses differ"
    assert list(e.tick(23, 8)) == list(o.tick(23, 8))
    _digests(e, o, "after tick 30")
    H.assert_same_state(e.store_state(), o.store_state(), "after tick 30")


@pytest.mark.parametrize("keep", ["1", "0"], ids=["kept", "copied_back"])
def test_corrupted_copies(monkeypatch, keep):
    """C5's shape with EXT corruption: a tick whose copy to a follower is
    corrupted goes to the list kernel (rejection: the follower's append
    skipped, AppendEntries false), and the next tick the follower catches up
    there. Round 6 (DevPlanes::sh_keep, the default): the group keeps its
    shared form through both — the rejecting follower's log is a prefix of the
    leader's and the 2K-slot shared ring still holds its window — so nothing
    is copied back; RAFTSTEP_SH_KEEP=0: the list kernel copies the group's
    shared entries back first (round 5's form)."""
    monkeypatch.setenv("RAFTSTEP_SH_KEEP", keep)
    e, o = _pair(monkeypatch, replicas=5, payload_crc=1, entries_per_tick=8, ring_depth=32,
                 corrupt_per_65536=300)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    e.diag_enable()
    t = 1
    for k in (8, 8, 16):
        assert list(e.tick(t, k)) == list(o.tick(t, k)), f"stats of ticks [{t}, {t + k})"
        t += k
    cls = e.diag_read()
    print("class counters:", cls)
    assert cls["lean_sh"] > 0 and cls["list_lag_catchup"] > 0, cls
    if keep == "1":
        assert cls["list_sh_kept"] > 0 and cls["list_sh_copied"] == 0, cls
    else:
        assert cls["list_sh_copied"] > 0 and cls["list_sh_kept"] == 0, cls
    # a digest mid-run (kept groups read from the shared ring, lagging ones too)
    _digests(e, o, f"after tick {t - 1}, before the host view")
    _digests(e, o, f"after tick {t - 1}")
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")


@pytest.mark.parametrize("E,K", [(8, 32), (16, 64)])
def test_several_lagging_followers(monkeypatch, E, K):
    """Round 6: with corruption at 3000/65536 per follower and tick, two or
    more followers of a group reject in the same tick (or one rejects again
    while it lags) ~1% of group-ticks; in the kept shared form their
    catch-ups copy nothing, so fast_group takes them all (case (ii) of
    main.go:353-360 per follower, one prevLogTerm ring read each) instead of
    deferring the group to the general kernel. E = 16: the shared ring in
    16-slot chunks (DevPlanes::sh_cs, the list kernel's wave-cooperative batch
    writes). Stats of every call, digests and the whole state against the
    oracle."""
    e, o = _pair(monkeypatch, replicas=5, payload_crc=1, entries_per_tick=E, ring_depth=K,
                 corrupt_per_65536=3000)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    e.diag_enable()
    t = 1
    for k in (8, 8, 16):
        assert list(e.tick(t, k)) == list(o.tick(t, k)), f"stats of ticks [{t}, {t + k})"
        t += k
        _digests(e, o, f"after tick {t - 1}")
    cls = e.diag_read()
    print("class counters:", cls)
    assert cls["list_sh_kept"] > 0 and cls["list_lag_catchup"] > 20 * max(1, cls["list_deferred"]), cls
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")


def test_forced_on_under_isolation_churn(monkeypatch):
    """RAFTSTEP_SH=2 (the A/B knob: shared entries under C4's leader-isolation
    churn too, with virtual suffixes and ring segment switches): every group
    leaves and re-enters the shared form through the list kernel's copy-back
    (the wave-cooperative one, round 6); statistics of every call, then
    digests and the whole state, equal the oracle's."""
    import bench
    monkeypatch.setenv("RAFTSTEP_SH", "2")
    wl = bench.WORKLOADS["C4"]
    kw = bench.engine_kwargs(wl, 7, 1 << 13, 0, wl["ring_depth"], 1, 0)
    kw["isolate_per_65536"] = 4 * wl["iso"][0]
    e, o = Engine(**kw), oracle.Oracle(**kw)
    assert e.features()["shared_entries"]
    e.diag_enable()
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    for k in (48, 20, 20, 20, 13, 30):
        assert list(e.tick(t, k)) == list(o.tick(t, k, threads=16)), f"stats of ticks [{t}, {t + k})"
        t += k
    cls = e.diag_read()
    assert cls["list_sh_copied"] > 100 and cls["lean_sh"] > 0 and cls["list_sh_entries"] > 0, cls
    _digests(e, o, f"after tick {t - 1}")
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
