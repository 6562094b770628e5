"""GPU: staged client values (raft_config.client_source = RAFT_CLIENT_STAGED,
raft_stage_values) against the CPU oracle fed the same buffer.

This is the drop-in LogReq path (main.go:87-93 -> 327-329): the caller, not
the engine's trace RNG, supplies every client value, so nothing the engine
stores can be regenerated — virtual suffixes are off and a returning stale
leader's catch-up is copied from the leader's ring (main.go:357,
GetLogsFrom) by the general kernel. Every kernel form that appends entries is
covered: the lean kernel (its whole-row, drifted, LXS and SXS writes), the
list kernel, the general kernel, the one-pass kernel, the fused steady
kernel, shared entries on and off, and the bench's full-size C2S / C4S lines
through oracle slices.
"""
import numpy as np
import pytest

import bench
import harness as H
import oracle
from raftstep import Engine, abi
from raftstep.engine import RaftError
from test_gpu_fullsize import SLICE, THREADS, check_slices, offsets

pytestmark = pytest.mark.gpu


def _stage(xs, seed, G, t, n, E, base=0):
    v = bench.staged_values(seed, base, G, t, n, E)
    for x in xs:
        x.stage_values(t, v)
    return v


def _run_both(e, o, calls, t, seed, E, G, full_at=(), stage_ahead=False):
    """Stages each call's values (or two calls' at once), runs the engine and
    the oracle, compares stats and digests after every call."""
    i = 0
    total = np.zeros(8, np.int64)
    while i < len(calls):
        n = calls[i]
        span = n + (calls[i + 1] if stage_ahead and i + 1 < len(calls) else 0)
        _stage([e, o], seed, G, t, span, E)
        for k in ([n, calls[i + 1]] if span != n else [n]):
            se = e.tick(t, k)
            so = o.tick(t, k, threads=THREADS)
            assert list(se) == list(so), f"stats [{t}, {t + k}): {list(se)} vs {list(so)}"
            total += se
            t += k
            de, _ = e.state_digest()
            do, _ = o.state_digest()
            bad = np.nonzero(de != do)[0]
            assert not bad.size, (f"after tick {t - 1}: {bad.size} digests differ, first {int(bad[0])}\n"
                                  f"engine:\n{e.nodelog(int(bad[0]))}oracle:\n{o.nodelog(int(bad[0]))}")
            if i in full_at:
                H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
            i += 1
    return t, total


FORMS = {
    "default": {},
    "no_shared_entries": {"RAFTSTEP_SH": "0"},
    "no_split": {"RAFTSTEP_SPLIT_STEADY": "0"},
    "one_pass": {"RAFTSTEP_TWO_PASS": "0"},
    "general": {"RAFTSTEP_FORCE_GENERAL": "1"},
    "general_lane": {"RAFTSTEP_FORCE_GENERAL": "1", "RAFTSTEP_GENERAL": "lane"},
}


@pytest.mark.parametrize("E", [1, 3])
@pytest.mark.parametrize("form", sorted(FORMS) + ["fused16"])
def test_staged_steady_matches_oracle(monkeypatch, form, E):
    """C2's shape (R=5, K=32, init_steady) at 2^17+300 groups — split steady
    tick, list skip, shared entries — with staged values through every tick
    form; stats and digests after every call, whole state at two points, and
    the leader's newest entries are the staged ones."""
    for k, v in FORMS.get(form, {}).items():
        monkeypatch.setenv(k, v)
    G = (1 << 17) + 300
    seed = 0x5EED0002
    kw = dict(replicas=5, groups=G, ring_depth=32, entries_per_tick=E, client_period=1, seed=seed,
              client_source=abi.CLIENT_STAGED)
    e = Engine(**kw, ticks_per_launch=16 if form == "fused16" else 1)
    o = oracle.Oracle(**kw)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    t, _ = _run_both(e, o, [5, 20, 20, 20], 1, seed, E, G, full_at=(0, 3), stage_ahead=(form == "default"))
    st = e.store_state_range(G - 5, 5)
    v = bench.staged_values(seed, G - 5, 5, t - 1, 1, E)
    for g in range(5):
        for r in range(5):
            assert [x for _, x in H.log_of(st, g, r, 32)][-E:] == [int(v[0, j, g]) for j in range(E)]


def test_staged_churn_matches_oracle_and_covers_the_classes():
    """C4's configuration (R=7, K=128, leader isolation, RAFT) on 2^16 groups
    with staged values, against ONE oracle over every group: elections, first
    rounds, stale leaders (their own appends stored, not virtual), returns
    (catch-up read from the primary's ring column by the list kernel), LXS /
    SXS / HWX, segment switches. Virtual suffixes are off in this mode."""
    wl = bench.WORKLOADS["C4S"]
    G = 1 << 16
    kw = bench.engine_kwargs(wl, 7, G, 0, wl["ring_depth"], 1, 0)
    assert kw["client_source"] == abi.CLIENT_STAGED
    e = Engine(**kw)
    assert e.features()["virtual_suffixes"] is False
    o = oracle.Oracle(**kw)
    e.diag_enable()
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    calls = [48, 5] + [20] * 20
    t, total = _run_both(e, o, calls, 0, wl["seed"], 1, G, full_at=(0, 10, len(calls) - 1))
    assert total[6] == 0
    assert t == 453
    cls = e.diag_read()
    print("class counters:", cls)
    need = ["lean_ssync", "lean_lxs", "lean_switch", "lean_hwx", "lean_sxs", "list_quiet", "list_isolated_leader",
            "list_election", "list_first_round", "list_stale", "list_window_start", "list_sxs_entered",
            "list_return", "list_return_trunc",   # (returns: catch-up read from the primary's column)
            "list_stale_moved", "lean_sxs_stale_in_row"]   # (moves: read from the stale leader's old slots)
    low = {k: cls[k] for k in need if cls[k] < 1000}
    assert not low, f"classes taken fewer than 1000 times: {low}\nall: {cls}"
    assert cls["list_return_vx"] == 0 and cls["lean_sxs_vx"] == 0 and cls["list_lxs_vx"] == 0
    assert cls["general_launches"] > 0


def test_staged_c5_with_corruption_matches_oracle():
    """C5's shape (E=64, CRC32C stamp + verify) with staged values and EXT
    corruption on: followers reject corrupted copies (main.go:148-149's
    append skipped, AppendEntries false) and catch up from the leader's ring.
    K = 256: a follower that missed one 64-entry batch is sent 128 entries
    with prevLogIndex 128 back, inside the window (with K = 128 that read is
    evicted after a single rejection: RAFT_F_RING_EVICTED, EXT)."""
    G = (1 << 14) + 77
    seed = 0x5EED0005
    kw = dict(replicas=5, groups=G, ring_depth=256, entries_per_tick=64, client_period=1, seed=seed,
              payload_crc=1, corrupt_per_65536=300, client_source=abi.CLIENT_STAGED)
    e = Engine(**kw)
    o = oracle.Oracle(**kw)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    e.diag_enable()
    _, total = _run_both(e, o, [3, 10, 10], 1, seed, 64, G, full_at=(2,))
    assert e.diag_read()["list_lag_catchup"] > 100
    # rejections happened (AppendEntries false); a fault needs 3 rejections of one follower in a row
    assert total[4] > 0 and total[6] <= 2


def test_staged_api_checks():
    G = 1024
    kw = dict(replicas=3, groups=G, ring_depth=16, entries_per_tick=2, client_period=1,
              client_source=abi.CLIENT_STAGED)
    e = Engine(**kw)
    e.init_steady(0, 0)
    with pytest.raises(RaftError) as x:
        e.tick(1, 4)                                   # nothing staged
    assert x.value.code == abi.RAFT_EINVAL and "not staged" in str(x.value)
    e.stage_values(1, np.zeros((4, 2, G), np.int64))
    e.tick(1, 4)
    with pytest.raises(RaftError):
        e.tick(5, 1)                                   # past the staged range
    with pytest.raises(RaftError):
        e.tick(0, 2)                                   # before it
    with pytest.raises(ValueError):
        e.stage_values(5, np.zeros((4, 1, G), np.int64))   # wrong E
    tr = Engine(replicas=3, groups=G)
    with pytest.raises(RaftError):
        tr.stage_values(0, np.zeros((1, 1, G), np.int64))  # a trace-RNG engine takes no values


def _run_sliced_staged(name, init, calls, state_at):
    wl = bench.WORKLOADS[name]
    R, G, E = wl.get("replicas", bench.R_DEFAULT), wl["groups"], wl["entries"]
    kw = bench.engine_kwargs(wl, R, G, 0, wl["ring_depth"], E, wl["crc"])
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
        e.stage_values(t, bench.staged_values(wl["seed"], 0, G, t, k, E))
        for o, off in zip(slices, offs):
            o.stage_values(t, bench.staged_values(wl["seed"], off, SLICE, t, k, E))
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


def test_c2s_as_benchmarked_full_size_slices():
    """bench.py --workload C2S: C2 (2^20 x R=5, E=1) with staged values through
    the bench's call structure; list skip and shared entries on."""
    cls, total, t = _run_sliced_staged("C2S", "steady", [5, 20, 20, 20], state_at=(0, 2, None))
    assert total[6] == 0 and total[0] == (1 << 20) * (t - 1)
    assert cls["ticks_list_skipped"] >= 40, cls


def test_c4s_as_benchmarked_full_size_slices():
    """bench.py --workload C4S: C4 (2^22 x R=7, K=128, leader isolation, RAFT)
    with staged values, 353 ticks past the 256-slot physical ring wrap."""
    wl = bench.WORKLOADS["C4S"]
    cls, total, t = _run_sliced_staged("C4S", "new", [wl["settle"], 5] + [20] * 15, state_at=(0, 8, None))
    assert total[6] == 0
    for k in ("list_election", "list_first_round", "list_stale", "lean_lxs", "lean_sxs"):
        assert cls[k] > 10000, (k, cls)
