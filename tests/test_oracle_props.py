"""Property tests (hypothesis) of the oracle on random seeded traces — REF
invariants read off main.go."""
import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from raftstep import abi

L = abi.LEADER


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**63 - 1), R=st.integers(1, 8), period=st.integers(0, 3),
       iso=st.sampled_from([0, 4000, 30000]), E=st.integers(1, 3))
def test_invariants_on_random_traces(oracle_mod, seed, R, period, iso, E):
    o = oracle_mod.Oracle(replicas=R, groups=24, client_period=period, entries_per_tick=E, seed=seed,
                          isolate_per_65536=iso, isolate_min_ticks=1, isolate_max_ticks=32, ring_depth=64)
    o.init_new_nodes(0)
    prev = o.store_state()
    prev_commit = {}
    for t in range(0, 120, 4):
        s = o.tick(t, 4)
        st_ = o.store_state()
        frozen = prev["fault"] != 0
        # frozen groups never change again
        for k in abi.STATE_FIELDS:
            a, b = prev[k][frozen], st_[k][frozen]
            assert (a == b).all(), k
        # terms never decrease; a fault never clears
        assert (st_["term"] >= prev["term"]).all()
        assert (st_["fault"][frozen] == prev["fault"][frozen]).all()
        # at most one leader per term in a group (votes are sticky bools, main.go:20, 160)
        for g in range(24):
            terms = st_["term"][g][st_["role"][g] == L]
            assert len(set(terms.tolist())) == len(terms), (g, st_["term"][g], st_["role"][g])
        # a leader's CommitIndex is monotone while it stays leader (main.go:387)
        for (g, r), c in list(prev_commit.items()):
            if st_["role"][g, r] == L and prev["role"][g, r] == L and prev["term"][g, r] == st_["term"][g, r]:
                assert st_["commit"][g, r] >= c
        prev_commit = {(g, r): st_["commit"][g, r] for g in range(24) for r in range(R) if st_["role"][g, r] == L}
        # matchIndex rows exist only for leaders; stats are non-negative
        assert (s >= 0).all()
        prev = st_


def test_steady_state_closed_form(oracle_mod):
    """KAT-1 generalised, run long: commit == last == N at the leader."""
    for R in (3, 5, 7):
        o = oracle_mod.Oracle(replicas=R, groups=10, client_period=1, seed=3)
        o.init_steady(-1, 0)
        s = o.tick(1, 200)
        st_ = o.store_state()
        assert (st_["last"] == 200).all()
        lead = st_["role"] == L
        assert (lead.sum(axis=1) == 1).all()
        assert (st_["commit"][lead] == 200).all() and (st_["commit"][~lead] == 199).all()
        assert list(s) == [2000, 0, 0, 2000 * (R - 1), 0, 0, 0, 2000]


def test_nodelog_format(oracle_mod):
    """nodelog line format of main.go:399-401."""
    o = oracle_mod.Oracle(replicas=3, groups=1)
    o.init_steady(1, 0)
    assert o.nodelog(0).splitlines() == ["[Server0:1:0:0][follower]", "[Server1:1:0:0][leader]",
                                         "[Server2:1:0:0][follower]"]
