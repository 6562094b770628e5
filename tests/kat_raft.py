"""Known-answer tests of the EXT RAFT-paper semantics mode (semantics=1),
hand-derived from the rules of Ongaro & Ousterhout's Figure 2 as restated in
oracle/raft_oracle.c (r_* functions). Same harness as tests/kat_cases.py: each
case takes make(cfg_kwargs) -> oracle or engine."""
from harness import C, F, L, ae_reqs, build_state, log_of, node, ops, vote_reqs
from raftstep import abi

K8 = 8
NONE = 0   # voted field in RAFT mode: votedFor + 1, 0 = none


def _impl(make, R, K=K8, **kw):
    return make(dict(replicas=R, ring_depth=K, groups=kw.pop("groups", 1), semantics=1, **kw))


def _op(impl, now, replica, kind, arg=0, group=0):
    r = impl.group_ops(now, ops([dict(group=group, replica=replica, kind=kind, arg=arg)]))[0]
    return int(r["status"]), int(r["fault"]), int(r["value"])


def _ae(impl, now, to, term, prev_idx=0, prev_term=0, lc=0, logs=(), group=0):
    reqs, ents = ae_reqs([dict(group=group, to=to, term=term, prev_log_index=prev_idx,
                               prev_log_term=prev_term, leader_commit=lc, logs=list(logs))])
    r = impl.append_entries(now, reqs, ents)[0]
    return int(r["success"]), int(r["match_index"]), int(r["term"]), int(r["fault"])


def _vr(impl, now, to, term, cand, lli=0, llt=0, group=0):
    q = vote_reqs([dict(group=group, to=to, term=term, candidate_id=cand)])
    q[0]["last_log_index"], q[0]["last_log_term"] = lli, llt
    r = impl.request_vote(now, q)[0]
    return int(r["vote_granted"]), int(r["term"]), int(r["fault"])


def _state(nodes, R, K=K8, next_=None):
    st = build_state([nodes], R, K)
    st["hwm"][0] = st["last"][0]
    for r, n in enumerate(nodes):
        if n["role"] == L:
            for p in range(R):
                st["next"][0, r, p] = 0 if p == r else (next_[p] if next_ else st["match"][0, r, p] + 1)
    return st


def raft01_election(make):
    """Timeout: Term++, votedFor = self; both peers (votedFor none, logs equally
    up to date) grant -> Leader with nextIndex = last+1, matchIndex = 0."""
    e = _impl(make, 3)
    e.init_new_nodes(0)
    assert _op(e, 6, 0, abi.OP_TIMEOUT) == (0, 0, 1)
    assert _op(e, 6, 0, abi.OP_CANDIDATE_ROUND) == (0, 0, 1)
    s = e.store_state()
    assert list(s["role"][0]) == [L, F, F] and list(s["term"][0]) == [1, 1, 1]
    assert list(s["voted"][0]) == [1, 1, 1]              # all voted for replica 0
    assert list(s["next"][0, 0]) == [0, 1, 1] and list(s["match"][0, 0]) == [0, 0, 0]


def raft02_up_to_date(make):
    """A candidate whose log is behind is refused, but its higher term is adopted
    and the vote forgotten."""
    e = _impl(make, 3)
    e.load_state(_state([node(F, 2, 2, [(1, 5), (2, 6)]), node(), node()], 3))
    assert _vr(e, 3, 0, term=3, cand=1, lli=5, llt=1) == (0, 3, 0)   # lastTerm 1 < 2
    s = e.store_state()
    assert s["term"][0, 0] == 3 and s["voted"][0, 0] == NONE
    assert _vr(e, 3, 0, term=3, cand=2, lli=2, llt=2) == (1, 3, 0)   # equal lastTerm, index >= 2
    assert e.store_state()["voted"][0, 0] == 3
    assert _vr(e, 3, 0, term=3, cand=1, lli=9, llt=9) == (0, 3, 0)   # already voted in term 3


def raft03_truncate(make):
    """Conflict at index 2 (term 1 vs 3): delete it and everything after, append
    the new entries; commit = min(LC, index of last new entry)."""
    e = _impl(make, 3)
    e.load_state(_state([node(F, 2, 0, [(1, 1), (1, 2), (2, 3)]), node(), node()], 3))
    assert _ae(e, 4, 0, term=3, prev_idx=1, prev_term=1, lc=5, logs=[(3, 7), (3, 8)]) == (1, 3, 3, 0)
    s = e.store_state()
    assert log_of(s, 0, 0, K8) == [(1, 1), (3, 7), (3, 8)] and s["commit"][0, 0] == 3
    assert s["hwm"][0, 0] == 3


def raft04_keep_matching(make):
    """Entries already present (same index and term) are not truncated."""
    e = _impl(make, 3)
    e.load_state(_state([node(F, 1, 0, [(1, 1), (1, 2)]), node(), node()], 3))
    assert _ae(e, 4, 0, term=1, prev_idx=0, prev_term=0, lc=9, logs=[(1, 1)]) == (1, 1, 1, 0)
    s = e.store_state()
    assert log_of(s, 0, 0, K8) == [(1, 1), (1, 2)] and s["commit"][0, 0] == 1


def raft05_consistency_failures(make):
    """Log too short -> false with hint = last; term mismatch at prevLogIndex ->
    false with hint = min(prevLogIndex-1, commitIndex); stale term -> false,
    timer untouched."""
    e = _impl(make, 3)
    e.load_state(_state([node(F, 1, 0, [(1, 1), (1, 2), (1, 3)], commit=1, deadline=40, timeout=11), node(),
                         node()], 3))
    assert _ae(e, 4, 0, term=1, prev_idx=5, prev_term=1) == (0, 3, 1, 0)
    assert _ae(e, 4, 0, term=1, prev_idx=2, prev_term=2) == (0, 1, 1, 0)    # min(1, commit 1)
    assert _ae(e, 4, 0, term=1, prev_idx=3, prev_term=2) == (0, 1, 1, 0)    # min(2, commit 1)
    assert e.store_state()["deadline"][0, 0] == 8 + 11      # both reset the timer (current leader)
    e2 = _impl(make, 3)
    e2.load_state(_state([node(F, 4, 0, [(4, 1)], deadline=40, timeout=11), node(), node()], 3))
    assert _ae(e2, 4, 0, term=3) == (0, 1, 4, 0)
    assert e2.store_state()["deadline"][0, 0] == 40


def raft06_backoff_and_commit(make):
    """Leader round: a follower whose log is short answers with its length; the
    leader backs nextIndex off to hint+1; the majority order statistic commits
    only an entry of the current term."""
    R = 3
    lead = node(L, 2, 1, [(1, 1), (1, 2), (2, 3), (2, 4)], commit=0, match=[0, 0, 0])
    e = _impl(make, R)
    e.load_state(_state([lead, node(F, 2, 1, [(1, 1)]), node(F, 2, 1, [(1, 1), (1, 2), (2, 3), (2, 4)])], R,
                        next_=[0, 4, 5]))
    st, fault, commit = _op(e, 5, 0, abi.OP_LEADER_ROUND)
    s = e.store_state()
    # peer 1: prev 3 > last 1 -> false, hint 1 -> next = min(3, 2) = 2; peer 2: heartbeat ok, match 4
    assert list(s["next"][0, 0]) == [0, 2, 5] and list(s["match"][0, 0]) == [0, 0, 4]
    assert commit == 4 and s["commit"][0, 0] == 4      # {4 (leader), 4, 0} -> N = 4, term 2 == current
    # next round brings peer 1 up to date
    _op(e, 6, 0, abi.OP_LEADER_ROUND)
    s = e.store_state()
    assert log_of(s, 0, 1, K8) == [(1, 1), (1, 2), (2, 3), (2, 4)] and list(s["match"][0, 0]) == [0, 4, 4]
    # current-term rule: majority on an old-term entry does not commit it
    e2 = _impl(make, R)
    e2.load_state(_state([node(L, 3, 1, [(1, 1), (2, 2)], match=[0, 2, 2]), node(F, 3, 1, [(1, 1), (2, 2)]),
                          node(F, 3, 1, [(1, 1), (2, 2)])], R, next_=[0, 3, 3]))
    assert _op(e2, 5, 0, abi.OP_LEADER_COMMIT) == (0, 0, 0)


def raft07_step_down(make):
    """Any higher term seen steps a leader/candidate down (votedFor cleared);
    a candidate accepts a same-term leader; no REF deadlocks exist here."""
    e = _impl(make, 3, groups=3)
    st = _state([node(L, 2, 1, [(2, 1)], match=[0, 0, 0]), node(F, 5, 0), node(F, 2, 1)], 3, next_=[0, 2, 2])
    g1 = _state([node(C, 3, 1, deadline=50), node(L, 3, 2), node(F, 3, 2)], 3, next_=[1, 0, 1])
    g2 = _state([node(L, 2, 1), node(C, 4, 2), node(F, 2, 1)], 3, next_=[0, 1, 1])
    for k in st:
        st[k] = __import__("numpy").concatenate([st[k], g1[k], g2[k]])
    e.load_state(st)
    _op(e, 3, 0, abi.OP_LEADER_ROUND, group=0)             # peer 1 answers with term 5
    s = e.store_state()
    assert s["role"][0, 0] == F and s["term"][0, 0] == 5 and s["voted"][0, 0] == NONE
    assert _ae(e, 3, 0, term=3, group=1) == (1, 0, 3, 0)   # candidate meets the term-3 leader
    s = e.store_state()
    assert s["role"][1, 0] == F and s["voted"][1, 0] == 1 and s["fault"][1] == 0
    assert _vr(e, 3, 0, term=4, cand=1, group=2) == (1, 4, 0)   # leader sees term 4 -> follower, grants
    s = e.store_state()
    assert s["role"][2, 0] == F and s["voted"][2, 0] == 2


def raft08_tick_steady(make):
    """Steady state (RAFT): after N ticks every log has N entries; leader
    commit N; followers N-1 (they learn the commit one round later)."""
    e = _impl(make, 5, groups=6, client_period=1)
    e.init_steady(-1, 0)
    N = 12
    s = e.tick(1, N)
    st = e.store_state()
    assert (st["last"] == N).all() and (st["fault"] == 0).all()
    lead = st["role"] == L
    assert (st["commit"][lead] == N).all() and (st["commit"][~lead] == N - 1).all()
    assert list(s) == [6 * N, 0, 0, 6 * 4 * N, 0, 0, 0, 6 * N]


ALL = [raft01_election, raft02_up_to_date, raft03_truncate, raft04_keep_matching, raft05_consistency_failures,
       raft06_backoff_and_commit, raft07_step_down, raft08_tick_steady]
