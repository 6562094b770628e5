"""The oracle's EXT RAFT-paper mode: hand-derived KATs plus the Raft safety
properties (election safety, log matching, state-machine safety) on random
churn traces."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import kat_raft
from raftstep import abi


def make_oracle(kw):
    import oracle
    return oracle.Oracle(**kw)


@pytest.mark.parametrize("case", kat_raft.ALL, ids=lambda f: f.__name__)
def test_oracle_raft_kat(case, oracle_mod):
    case(make_oracle)


def check_raft_safety(snapshots, K):
    """snapshots: list of store_state dicts over time (one group set)."""
    leaders_by_term = {}
    committed = {}
    for s in snapshots:
        G, R = s["role"].shape
        for g in range(G):
            for r in range(R):
                if s["role"][g, r] == abi.LEADER:
                    key = (g, int(s["term"][g, r]))
                    assert leaders_by_term.setdefault(key, r) == r, f"two leaders in term {key}"
            # log matching within the ring windows
            for a in range(R):
                for b in range(a + 1, R):
                    lo = max(1, int(s["hwm"][g, a]) - K + 1, int(s["hwm"][g, b]) - K + 1)
                    hi = min(int(s["last"][g, a]), int(s["last"][g, b]))
                    same = [i for i in range(lo, hi + 1)
                            if s["log_term"][g, a, (i - 1) % K] == s["log_term"][g, b, (i - 1) % K]]
                    if same:
                        top = max(same)
                        for i in range(lo, top + 1):
                            ea = (s["log_term"][g, a, (i - 1) % K], s["log_value"][g, a, (i - 1) % K])
                            eb = (s["log_term"][g, b, (i - 1) % K], s["log_value"][g, b, (i - 1) % K])
                            assert ea == eb, f"log matching broken g={g} {a}/{b} at {i}"
            # state machine safety: a committed index never changes content
            for r in range(R):
                lo = max(1, int(s["hwm"][g, r]) - K + 1)
                for i in range(lo, min(int(s["commit"][g, r]), int(s["last"][g, r])) + 1):
                    e = (int(s["log_term"][g, r, (i - 1) % K]), int(s["log_value"][g, r, (i - 1) % K]))
                    assert committed.setdefault((g, i), e) == e, f"committed entry {i} of group {g} changed"


@settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**62), R=st.sampled_from([3, 5, 7]), iso=st.sampled_from([8000, 30000, 60000]))
def test_raft_safety_under_churn(oracle_mod, seed, R, iso):
    K = 64
    o = oracle_mod.Oracle(replicas=R, groups=12, ring_depth=K, client_period=1, seed=seed, semantics=1,
                          isolate_per_65536=iso, isolate_min_ticks=2, isolate_max_ticks=32)
    o.init_new_nodes(0)
    snaps = []
    for t in range(0, 240, 6):
        o.tick(t, 6)
        snaps.append(o.store_state())
    # the only possible fault: a follower more than K entries behind (no
    # InstallSnapshot in a fixed ring) — RING_EVICTED; everyone else progresses
    f = snaps[-1]["fault"]
    assert set(f.tolist()) <= {0, abi.F_RING_EVICTED}
    check_raft_safety(snaps, K)
    assert (snaps[-1]["commit"].max(axis=1)[f == 0] > 100).all()
