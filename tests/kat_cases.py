"""Known-answer tests, hand-derived from eastwd/raft-sample main.go
(SURVEY.md Appendix B). Each case takes `make(cfg_kwargs) -> impl` where impl
is the oracle (CPU, tests/test_oracle_kat.py) or the HIP engine (GPU,
tests/test_gpu_kat.py), so the same expectations pin both.

Expected values below are derived from the reference text, not from either
implementation; each case cites the lines it exercises.
"""
import numpy as np

import harness
from harness import C, F, L, ae_reqs, build_state, log_of, node, ops, vote_reqs
from raftstep import abi

K8 = 8


def _impl(make, R, K=K8, **kw):
    return make(dict(replicas=R, ring_depth=K, groups=kw.pop("groups", 1), **kw))


def _op(impl, now, replica, kind, arg=0, group=0):
    r = impl.group_ops(now, ops([dict(group=group, replica=replica, kind=kind, arg=arg)]))[0]
    return int(r["status"]), int(r["fault"]), int(r["value"])


def _ae(impl, now, to, term, prev_idx=0, prev_term=0, lc=0, logs=(), group=0):
    reqs, ents = ae_reqs([dict(group=group, to=to, term=term, prev_log_index=prev_idx,
                               prev_log_term=prev_term, leader_commit=lc, logs=list(logs))])
    r = impl.append_entries(now, reqs, ents)[0]
    return int(r["success"]), int(r["match_index"]), int(r["fault"])


def _vr(impl, now, to, term, group=0):
    r = impl.request_vote(now, vote_reqs([dict(group=group, to=to, term=term)]))[0]
    return int(r["vote_granted"]), int(r["fault"])


def kat01_election(make):
    """KAT-1: 3 x NewNode; S0's timer fires (main.go:171-177), its vote round
    (main.go:253-284) gets both grants (main.go:157-170) -> Leader."""
    e = _impl(make, 3)
    e.init_new_nodes(0)
    s0 = e.store_state()
    assert (s0["role"] == F).all() and (s0["term"] == 0).all() and (s0["voted"] == 0).all()
    st, fault, term = _op(e, 5, 0, abi.OP_TIMEOUT)
    assert (st, fault, term) == (0, 0, 1)
    st, fault, won = _op(e, 5, 0, abi.OP_CANDIDATE_ROUND)
    assert (st, fault, won) == (0, 0, 1)
    s = e.store_state()
    assert list(s["role"][0]) == [L, F, F]
    assert list(s["term"][0]) == [1, 1, 1]
    assert list(s["voted"][0]) == [1, 1, 1]
    assert list(s["match"][0, 0]) == [0, 0, 0]
    # grants reset the followers' timers with their own d (main.go:164-167)
    assert list(s["deadline"][0, 1:]) == [10 + s0["timeout"][0, 1], 10 + s0["timeout"][0, 2]]
    return e


def kat02_heartbeat_empty(make):
    """KAT-2: empty-log heartbeat (main.go:364-371); followers skip the checks
    (last == 0, main.go:135); histogram {0:2} but 0 > CommitIndex fails (main.go:387)."""
    e = kat01_election(make)
    st, fault, commit = _op(e, 6, 0, abi.OP_LEADER_ROUND)
    assert (st, fault, commit) == (0, 0, 0)
    s = e.store_state()
    assert list(s["last"][0]) == [0, 0, 0] and list(s["commit"][0]) == [0, 0, 0]
    assert list(s["match"][0, 0]) == [0, 0, 0]
    return e


def kat03_first_entry(make):
    """KAT-3: client append (main.go:327-329) then NextIndex==1 -> whole log,
    PrevLogIndex 0 (main.go:343-351); both peers at 1 -> leader commit 1."""
    e = kat02_heartbeat_empty(make)
    A = 0x1234
    assert _op(e, 7, 0, abi.OP_CLIENT_APPEND, A) == (0, 0, 1)
    assert _op(e, 7, 0, abi.OP_LEADER_ROUND) == (0, 0, 1)
    s = e.store_state()
    for r in range(3):
        assert log_of(s, 0, r, K8) == [(1, A)]
    assert list(s["match"][0, 0]) == [0, 1, 1]
    assert list(s["commit"][0]) == [1, 0, 0]
    return e


def kat04_commit_propagates(make):
    """KAT-4: heartbeat PrevLogIndex=1, PrevLogTerm=Term (main.go:369);
    followers' CommitIndex = min(LC=1, len+1=2) = 1 (main.go:151-152)."""
    e = kat03_first_entry(make)
    assert _op(e, 8, 0, abi.OP_LEADER_ROUND) == (0, 0, 1)
    s = e.store_state()
    assert list(s["commit"][0]) == [1, 1, 1]
    assert list(s["last"][0]) == [1, 1, 1]
    return e


def kat05_suffix(make):
    """KAT-5: NextIndex 2 <= LastApplied 2 -> GetLogsFrom(2), PrevLogTerm =
    GetLog(MatchIndex=1).Term (main.go:353-360); match {2,2} -> commit 2."""
    e = kat04_commit_propagates(make)
    B = 0x5678
    assert _op(e, 9, 0, abi.OP_CLIENT_APPEND, B) == (0, 0, 2)
    assert _op(e, 9, 0, abi.OP_LEADER_ROUND) == (0, 0, 2)
    s = e.store_state()
    for r in range(3):
        assert log_of(s, 0, r, K8) == [(1, 0x1234), (1, B)]
    assert list(s["match"][0, 0]) == [0, 2, 2]
    assert list(s["commit"][0]) == [2, 1, 1]   # followers got LC=1 in this round


def kat06_commit_plus_one(make):
    """KAT-6: CommitIndex = min(LC=9, len(Log)+1=3) = 3 > len (main.go:152)."""
    e = _impl(make, 3)
    e.load_state(build_state([[node(F, 1, 1, [(1, 11), (1, 12)]), node(F, 1, 1), node(F, 1, 1)]], 3, K8))
    assert _ae(e, 3, 0, term=1, prev_idx=2, prev_term=1, lc=9) == (1, 2, 0)
    s = e.store_state()
    assert s["commit"][0, 0] == 3 and s["last"][0, 0] == 2 and s["term"][0, 0] == 1


def _leader_commit_case(make, R, match, commit):
    nodes = [node(F, 1, 1) for _ in range(R)]
    nodes[0] = node(L, 1, 1, [(1, i) for i in range(max(match + [commit, 1]))], commit=commit,
                    match=[0] + list(match))
    e = _impl(make, R)
    e.load_state(build_state([nodes], R, K8))
    st, fault, c = _op(e, 3, 0, abi.OP_LEADER_COMMIT)
    assert (st, fault) == (0, 0)
    s = e.store_state()
    assert s["commit"][0, 0] == c
    return c


def kat07_10_commit_rule(make):
    """KAT-7..10: exact-value histogram over peers, leader excluded, 2*count > N
    and i > CommitIndex (main.go:381-391) — not the majority order statistic."""
    assert _leader_commit_case(make, 5, [3, 3, 2, 2], 0) == 0          # KAT-7 (textbook: 3)
    assert _leader_commit_case(make, 5, [3, 3, 3, 2], 0) == 3          # KAT-8
    assert _leader_commit_case(make, 5, [1, 1, 1, 1], 2) == 2          # KAT-9 (monotone)
    assert _leader_commit_case(make, 7, [4, 4, 4, 3, 3, 3], 0) == 0    # KAT-10a
    assert _leader_commit_case(make, 7, [4, 4, 4, 4, 3, 3], 0) == 4    # KAT-10b
    assert _leader_commit_case(make, 2, [1], 0) == 0                   # R=2 never commits
    assert _leader_commit_case(make, 4, [3, 3, 3], 0) == 3             # R=4 needs all 3 peers
    assert _leader_commit_case(make, 4, [3, 3, 2], 0) == 0


def kat11_panic_getlog(make):
    """KAT-11: a new leader's first heartbeat (PrevLogIndex 0) to a follower
    with entries: GetLog(0) panics (main.go:142 -> 404) -> group frozen."""
    e = _impl(make, 3)
    e.load_state(build_state([[node(F, 1, 1, [(1, 5), (1, 6)], deadline=40, timeout=17),
                               node(F, 1, 1), node(F, 1, 1)]], 3, K8))
    ok, match, fault = _ae(e, 4, 0, term=2, prev_idx=0, prev_term=2)
    assert ok == 0 and fault == abi.F_PANIC_GETLOG
    s = e.store_state()
    assert s["fault"][0] == abi.F_PANIC_GETLOG
    assert s["deadline"][0, 0] == 8 + 17      # timer was reset before the panic (main.go:124-127)
    assert s["term"][0, 0] == 1 and s["last"][0, 0] == 2
    # frozen: further messages change nothing
    assert _vr(e, 5, 1, 9) == (0, abi.F_PANIC_GETLOG)
    assert e.store_state()["term"][0, 1] == 1


def kat12_stale_term(make):
    """KAT-12: r.Term < Term -> false with MatchIndex=LastApplied (main.go:129-133);
    the timer is still reset (main.go:124-127)."""
    e = _impl(make, 3)
    e.load_state(build_state([[node(F, 5, 0, [(5, 1)], deadline=3, timeout=21), node(), node()]], 3, K8))
    assert _ae(e, 7, 0, term=3) == (0, 1, 0)
    s = e.store_state()
    assert s["term"][0, 0] == 5 and s["deadline"][0, 0] == 14 + 21


def kat13_candidate_steps_down(make):
    """KAT-13: candidate gets AE with r.Term >= Term: Success with MatchIndex =
    LastApplied WITHOUT appending, -> Follower, Voted, Term (main.go:204-216)."""
    e = _impl(make, 3)
    e.load_state(build_state([[node(C, 3, 1, [(2, 7)], deadline=50, timeout=11), node(), node()]], 3, K8))
    ok, match, fault = _ae(e, 6, 0, term=3, prev_idx=0, prev_term=3, lc=4, logs=[(3, 1), (3, 2)])
    assert (ok, match, fault) == (1, 1, 0)
    s = e.store_state()
    assert s["role"][0, 0] == F and s["voted"][0, 0] == 1 and s["term"][0, 0] == 3
    assert s["last"][0, 0] == 1 and s["commit"][0, 0] == 0
    assert log_of(s, 0, 0, K8) == [(2, 7)]
    assert 10 <= s["timeout"][0, 0] <= 29                      # new FollowerRun timer (main.go:114)
    assert s["deadline"][0, 0] == 12 + s["timeout"][0, 0]
    # leader side: the candidate's MatchIndex becomes its LastApplied (main.go:375-377)
    e2 = _impl(make, 3)
    e2.load_state(build_state([[node(L, 3, 1, [(3, i) for i in range(5)], match=[0, 0, 0]),
                                node(C, 3, 1, [(2, 9)]), node(F, 3, 1)]], 3, K8))
    assert _op(e2, 2, 0, abi.OP_LEADER_ROUND) == (0, 0, 0)    # histogram {1:1, 5:1}
    s = e2.store_state()
    assert list(s["match"][0, 0]) == [0, 1, 5]
    assert s["role"][0, 1] == F and s["last"][0, 1] == 1
    assert log_of(s, 0, 2, K8) == [(3, i) for i in range(5)]


def kat14_leader_steps_down(make):
    """KAT-14: leader gets AE with higher term: Success, MatchIndex 0,
    -> Follower with Voted=false (main.go:312-320)."""
    e = _impl(make, 3)
    e.load_state(build_state([[node(F, 2, 1), node(L, 2, 1, [(2, 3)], match=[1, 0, 1]), node(F, 2, 1)]], 3, K8))
    assert _ae(e, 3, 1, term=3, prev_idx=0, prev_term=3) == (1, 0, 0)
    s = e.store_state()
    assert s["role"][0, 1] == F and s["voted"][0, 1] == 0 and s["term"][0, 1] == 3
    assert list(s["match"][0, 1]) == [0, 0, 0]
    assert _ae(e, 3, 0, term=3) == (1, 0, 0)   # sanity: plain follower heartbeat
    e2 = _impl(make, 3)
    e2.load_state(build_state([[node(F, 2, 1), node(L, 2, 1, match=[0, 0, 0]), node(F, 2, 1)]], 3, K8))
    assert _ae(e2, 3, 1, term=2) == (0, 0, 0)  # equal term -> false (main.go:323-326)
    assert e2.store_state()["role"][0, 1] == L


def kat15_sticky_vote(make):
    """KAT-15: Voted is a sticky bool: VoteRequest{T=2} rejected, no timer reset
    (main.go:160-162)."""
    e = _impl(make, 3)
    e.load_state(build_state([[node(L, 1, 1), node(F, 1, 1, deadline=33), node(F, 1, 0, deadline=35, timeout=12)]],
                             3, K8))
    assert _vr(e, 9, 1, 2) == (0, 0)
    s = e.store_state()
    assert s["term"][0, 1] == 1 and s["deadline"][0, 1] == 33
    # a follower that has not voted grants, adopts the term and resets its timer (main.go:164-170)
    assert _vr(e, 9, 2, 2, group=0) == (1, 0)
    s = e.store_state()
    assert s["term"][0, 2] == 2 and s["voted"][0, 2] == 1 and s["deadline"][0, 2] == 18 + 12


def kat16_prev_term_mismatch(make):
    """KAT-16: heartbeat PrevLogTerm = current Term (main.go:369) against an
    older-term entry -> false (main.go:142-145); CommitIndex unchanged."""
    e = _impl(make, 3)
    e.load_state(build_state([[node(F, 4, 1, [(3, 1)]), node(), node()]], 3, K8))
    assert _ae(e, 2, 0, term=4, prev_idx=1, prev_term=4, lc=1) == (0, 1, 0)
    s = e.store_state()
    assert s["commit"][0, 0] == 0 and s["last"][0, 0] == 1


def kat17_deadlocks(make):
    """Candidate rejecting a same-term VoteRequest answers into its OWN VRes
    (main.go:242): the requester blocks at main.go:265; a leader has no VReq case
    (main.go:308) — both freeze the group with a fault code."""
    e = _impl(make, 3, groups=3)
    e.load_state(build_state([
        [node(C, 2, 1, deadline=5, timeout=13), node(C, 2, 1), node()],
        [node(L, 2, 1), node(), node()],
        [node(C, 2, 1), node(F, 2, 1), node(C, 1, 1, timeout=12)],
    ], 3, K8))
    r = e.request_vote(10, vote_reqs([dict(group=0, to=0, term=2), dict(group=1, to=0, term=5)]))
    assert list(r["fault"]) == [abi.F_DEADLOCK_VRES, abi.F_DEADLOCK_LEADER_VREQ]
    assert list(r["vote_granted"]) == [0, 0]
    s = e.store_state()
    assert s["deadline"][0, 0] == 20 + 13           # main.go:243-246
    # candidate with lower term grants to a higher-term candidate and steps down (main.go:227-238)
    st, fault, won = _op(e, 10, 0, abi.OP_CANDIDATE_ROUND, group=2)
    s = e.store_state()
    assert (st, fault) == (0, 0)
    assert s["role"][2, 2] == F and s["term"][2, 2] == 2 and s["voted"][2, 2] == 1
    # replica 1 (sticky Voted) rejected, replica 2 granted: count 2, 2*2 > 3 -> Leader
    assert won == 1 and s["role"][2, 0] == L


def kat18_edge_replicas(make):
    """R=1 is elected by its own vote (2*1 > 1, main.go:273) and never commits
    (empty histogram); R=2 can never commit (2*1 > 2 false)."""
    e = _impl(make, 1)
    e.init_new_nodes(0)
    assert _op(e, 20, 0, abi.OP_TIMEOUT) == (0, 0, 1)
    assert _op(e, 20, 0, abi.OP_CANDIDATE_ROUND) == (0, 0, 1)
    assert _op(e, 20, 0, abi.OP_CLIENT_APPEND, 5) == (0, 0, 1)
    assert _op(e, 20, 0, abi.OP_LEADER_ROUND) == (0, 0, 0)
    e2 = _impl(make, 2)
    e2.init_new_nodes(0)
    assert _op(e2, 20, 1, abi.OP_TIMEOUT)[2] == 1
    assert _op(e2, 20, 1, abi.OP_CANDIDATE_ROUND) == (0, 0, 1)   # 2*2 > 2
    for t in range(3):
        _op(e2, 21 + t, 1, abi.OP_CLIENT_APPEND, t)
        assert _op(e2, 21 + t, 1, abi.OP_LEADER_ROUND) == (0, 0, 0)
    s = e2.store_state()
    assert list(s["last"][0]) == [3, 3] and s["match"][0, 1, 0] == 3


def kat19_role_checks(make):
    """Node steps are only run by the role whose loop has them (Run,
    main.go:98-109): a follower has no leader round etc."""
    e = _impl(make, 3)
    e.init_new_nodes(0)
    assert _op(e, 1, 0, abi.OP_LEADER_ROUND)[0] == abi.RAFT_EINVAL
    assert _op(e, 1, 0, abi.OP_CANDIDATE_ROUND)[0] == abi.RAFT_EINVAL
    assert _op(e, 1, 0, abi.OP_CLIENT_APPEND, 1)[0] == abi.RAFT_EINVAL
    assert _op(e, 1, 0, abi.OP_LEADER_COMMIT)[0] == abi.RAFT_EINVAL


def kat20_ext_limits(make):
    """EXT rules shared by engine and oracle: GetLog below the ring window
    faults RING_EVICTED; int32 overflow faults OVERFLOW."""
    e = _impl(make, 3, K=4, groups=2)
    I32 = 2**31 - 1
    e.load_state(build_state([
        [node(F, 1, 1, [(1, i) for i in range(10)]), node(), node()],
        [node(F, I32, 0), node(), node()],
    ], 3, 4))
    assert _ae(e, 1, 0, term=1, prev_idx=6, prev_term=1)[2] == abi.F_RING_EVICTED
    assert _op(e, 1, 0, abi.OP_TIMEOUT, group=1)[1] == abi.F_OVERFLOW
    e2 = _impl(make, 3, K=4)
    e2.load_state(build_state([[node(F, 1, 1, [(1, i) for i in range(10)]), node(), node()]], 3, 4))
    assert _ae(e2, 1, 0, term=1, prev_idx=7, prev_term=1, logs=[(1, 77)] * 6) == (1, 16, 0)
    s = e2.store_state()
    assert log_of(s, 0, 0, 4) == [(1, 77)] * 4


def kat21_tick_election(make):
    """Tick model from NewNode: the replica with the earliest (deadline, id)
    times out first, at tick ceil(d/2) (1 tick = 2 s, main.go:394), and wins
    with every vote; the grants reset the other timers (main.go:164-167)."""
    e = _impl(make, 3, groups=4, client_period=0)
    e.init_new_nodes(0)
    s0 = e.store_state()
    stats = e.tick(1, 15)
    s = e.store_state()
    for k, v in dict(elections_won=4, term_bumps=4, votes_granted=8, faults=0).items():
        assert stats[abi.STAT_NAMES.index(k)] == v, k
    for g in range(4):
        d = s0["deadline"][g]
        assert 5 <= int(np.ceil(d.min() / 2)) <= 15
        winner = int(np.argmin(d))      # argmin keeps the lowest id on ties
        assert list(s["role"][g]) == [L if r == winner else F for r in range(3)], (g, d)
        assert (s["term"][g] == 1).all() and (s["voted"][g] == 1).all()


def kat22_tick_steady(make):
    """Tick model, steady state (KAT-1 generalised, R=5, one entry per tick):
    after N ticks every log has N entries, leader commit N, followers N-1."""
    e = _impl(make, 5, groups=8, client_period=1, entries_per_tick=1)
    e.init_steady(0, 0)
    N = 20
    stats = e.tick(1, N)
    s = e.store_state()
    assert (s["last"] == N).all()
    assert (s["commit"][:, 0] == N).all() and (s["commit"][:, 1:] == N - 1).all()
    assert (s["fault"] == 0).all()
    exp = dict(committed=8 * N, ae_ok=8 * 4 * N, leader_groups=8 * N)
    for k, v in exp.items():
        assert stats[abi.STAT_NAMES.index(k)] == v, k
    for k in ("elections_won", "term_bumps", "ae_fail", "faults"):
        assert stats[abi.STAT_NAMES.index(k)] == 0, k


def kat23_crc_reject(make):
    """EXT (config C5): with payload CRC32C on, a follower whose copy of the
    last entry arrives with a flipped bit rejects the whole AppendEntries
    (nothing appended; its timer was already reset, main.go:124-127); the
    leader's MatchIndex does not move (main.go:375) and nothing commits."""
    e = _impl(make, 3, K=16, payload_crc=1, corrupt_per_65536=65536, client_period=1)
    e.init_steady(0, 0)
    s = e.tick(1, 3)
    st = e.store_state()
    assert list(st["last"][0]) == [3, 0, 0] and list(st["commit"][0]) == [0, 0, 0]
    assert s[abi.STAT_NAMES.index("ae_fail")] == 6 and s[abi.STAT_NAMES.index("ae_ok")] == 0
    assert st["log_crc"][0, 0, 0] == harness.entry_crc(1, st["log_value"][0, 0, 0])
    e2 = _impl(make, 3, K=16, payload_crc=1, corrupt_per_65536=0, client_period=1)
    e2.init_steady(0, 0)
    e2.tick(1, 3)
    st2 = e2.store_state()
    assert list(st2["last"][0]) == [3, 3, 3] and list(st2["commit"][0]) == [3, 2, 2]
    assert (st2["log_crc"][0, :, :3] == st2["log_crc"][0, 0, :3]).all()


ALL = [kat01_election, kat02_heartbeat_empty, kat03_first_entry, kat04_commit_propagates, kat05_suffix,
       kat06_commit_plus_one, kat07_10_commit_rule, kat11_panic_getlog, kat12_stale_term,
       kat13_candidate_steps_down, kat14_leader_steps_down, kat15_sticky_vote, kat16_prev_term_mismatch,
       kat17_deadlocks, kat18_edge_replicas, kat19_role_checks, kat20_ext_limits, kat21_tick_election,
       kat22_tick_steady, kat23_crc_reject]
