"""GPU: the pipelined tick (engine.cpp raft_engine::pipeline) and the
overlapped general kernel against the oracle, across the call and window
shapes where they hand groups from one kernel to another: calls of 1, 2, 7
and 20 ticks, general-kernel windows of 1, 3 and 8 ticks (window ends inside a
call, at a call's end, on consecutive ticks), pipeline on and off, in line
and overlapped general kernel (overlapping 1, 2 or 3 ticks), the pipelined
tick on ping-pong streams (default) or lean / list streams
(RAFTSTEP_PINGPONG=0), calls with and without statistics (the
stats-less form skips the per-tick records and the list kernel's second-step
records). Workload: C4's configuration (leader
isolation, RAFT; elections, first rounds, returns, deferrals) on 2^13 groups
at four times C4's churn, and REF semantics with hashed isolation (faults);
stats per call and per-group digests after every call, the whole canonical
state at the end. Anchors: main.go:171-177, 253-284, 309-320, 121-156."""
import numpy as np
import pytest

import bench
import harness as H
import oracle
from raftstep import Engine

pytestmark = pytest.mark.gpu
CALLS = [48, 1, 2, 7, 20, 1, 20, 2, 7, 20]


def _kw(sem):
    wl = bench.WORKLOADS["C4" if sem == 1 else "C4REF"]
    kw = bench.engine_kwargs(wl, 7, 1 << 13, 0, wl["ring_depth"], 1, 0)
    kw["isolate_per_65536"] = 4 * wl["iso"][0]
    if sem == 0:
        kw["isolate_leader"] = 0
    return kw


@pytest.mark.parametrize("sem", [1, 0])
@pytest.mark.parametrize("pipeline,overlap,slow_every,stats,pingpong",
                         [("1", "1", "8", True, "1"), ("1", "1", "3", True, "1"), ("1", "1", "1", True, "1"),
                          ("1", "0", "3", True, "1"), ("0", "1", "3", True, "1"), ("0", "0", "8", True, "1"),
                          ("1", "1", "8", False, "1"), ("1", "1", "3", False, "1"), ("0", "1", "3", False, "1"),
                          ("1", "2", "8", True, "1"), ("1", "2", "3", True, "1"), ("1", "3", "8", True, "1"),
                          ("1", "2", "1", True, "1"), ("0", "2", "3", True, "1"), ("1", "2", "8", False, "1"),
                          ("1", "2", "8", True, "0"), ("1", "1", "3", True, "0"), ("1", "2", "1", True, "0"),
                          ("1", "2", "3", False, "0"), ("1", "3", "3", True, "1"), ("1", "3", "1", True, "0"),
                          ("1", "3", "8", False, "1"), ("0", "3", "3", True, "1")])
def test_pipelined_tick_matches_oracle(monkeypatch, sem, pipeline, overlap, slow_every, stats, pingpong):
    monkeypatch.setenv("RAFTSTEP_PIPELINE", pipeline)
    monkeypatch.setenv("RAFTSTEP_PINGPONG", pingpong)
    monkeypatch.setenv("RAFTSTEP_DEBUG_PIPE", "1")
    monkeypatch.setenv("RAFTSTEP_OVERLAP_GENERAL", overlap)
    monkeypatch.setenv("RAFTSTEP_SLOW_EVERY", slow_every)
    kw = _kw(sem)
    e, o = Engine(**kw), oracle.Oracle(**kw)
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    for k in CALLS:
        se = e.tick(t, k, stats=stats)
        so = o.tick(t, k, threads=16)
        if stats:
            assert list(se) == list(so), f"stats of ticks [{t}, {t + k})"
        t += k
        de, _ = e.state_digest()
        do, _ = o.state_digest()
        bad = np.nonzero(de != do)[0]
        assert not bad.size, f"after tick {t - 1}: {bad.size} digests differ, first group {int(bad[0])}\n" \
                             f"engine:\n{e.nodelog(int(bad[0]))}oracle:\n{o.nodelog(int(bad[0]))}"
    H.assert_same_state(e.store_state(), o.store_state(), f"after tick {t - 1}")
    e.close()
    o.close()
