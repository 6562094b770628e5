"""Tick-level known-answer tests: whole fused ticks (raft_tick / the oracle's
tick), starting from hand-built states with chosen deadlines and timer
durations, with every expected value derived BY HAND from the main.go text
(eastwd/raft-sample) and the documented tick model (SURVEY.md Appendix A.3:
per tick, 1. client append to every Leader, 2. rounds of every Leader /
Candidate in ascending id, each message through the receiver's handler,
3. expired election timers in (deadline, id) order, each new candidate
running its vote round at once; now = tick * 2 s, main.go:394).

Neither implementation is consulted for an expected value. Where the
reference draws a random number (rand.Intn at a role entry, main.go:114,
194; rand.Int for a client value, main.go:92) the draw is the trace's
counter RNG, restated below from its definition (splitmix64 keyed by seed,
global group id, replica, stream, tick) and pinned by
tests/golden/rng_vectors.json.

Cases (REF semantics, no isolation, no CRC):
  T1  R=3: NewNode-like start -> S0's timer fires -> election -> first
      entries replicated and committed (main.go:171-177, 253-284, 157-170,
      327-329, 341-360, 121-156, 381-391).
  T2  R=5: a leader's heartbeat at a higher term steps a stale leader down
      (main.go:309-320), the next tick's whole-log AppendEntries (PrevLogIndex
      0, main.go:343-351) panics at its GetLog (main.go:142 -> 404).
  T3  R=3: election, then the new leader's first contact with followers that
      hold entries: GetLog(0) panics (KAT-11 through the fused tick).
  T4  R=5: two candidates of one term: the second rejects the first's
      VoteRequest into its own VRes (main.go:242), the requester blocks
      (main.go:265) and the group freezes mid-round; the replica after it
      never receives the request.
"""
from harness import F, C, L, build_state, node

MASK64 = (1 << 64) - 1
ST_VALUE, ST_TIMER_F, ST_TIMER_C = 1, 2, 3
K = 8


def sm64(x):
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
    return x ^ (x >> 31)


def trace_rng(seed, gid, replica, stream, tick):
    k = sm64(seed ^ sm64(gid))
    h = sm64(k ^ ((stream << 32) | replica))
    return sm64(h ^ tick)


def client_value(seed, gid, replica, tick, e=0):   # rand.Int() (main.go:92)
    return sm64(trace_rng(seed, gid, replica, ST_VALUE, tick) ^ e) >> 1


def draw_f(seed, gid, replica, tick):   # rand.Intn(20)+10 (main.go:114)
    return 10 + ((trace_rng(seed, gid, replica, ST_TIMER_F, tick) >> 32) % 20)


def draw_c(seed, gid, replica, tick):   # rand.Intn(4)+10 (main.go:194)
    return 10 + ((trace_rng(seed, gid, replica, ST_TIMER_C, tick) >> 32) % 4)


def zero_stats():
    return dict(committed=0, elections_won=0, term_bumps=0, ae_ok=0, ae_fail=0, votes_granted=0, faults=0,
                leader_groups=0)


def stats(**kw):
    s = zero_stats()
    s.update(kw)
    return s


def case_t1():
    seed, gid = 0x7E57_0001, 0
    R = 3
    cfg = dict(replicas=R, groups=1, ring_depth=K, client_period=1, entries_per_tick=1, seed=seed)
    # NewNode (main.go:59-76): Follower, Term 0, not Voted, empty log; timers
    # chosen: S0 expires at 4 s, S1/S2 far later; d = 20 s for everyone
    start = [node(F, 0, 0, deadline=4, timeout=20), node(F, 0, 0, deadline=100, timeout=20),
             node(F, 0, 0, deadline=100, timeout=20)]
    per_tick = [
        zero_stats(),                 # tick 0, now 0: nothing due
        zero_stats(),                 # tick 1, now 2
        # tick 2, now 4: S0's timer.C (main.go:171-177): Term 1, Candidate,
        # d_C drawn (194); its round (253-284) at once: S1 and S2 grant
        # (157-170: 1 >= 0, not Voted; timer.Reset -> 4+20); 2*3 > 3 -> Leader
        stats(elections_won=1, term_bumps=1, votes_granted=2, leader_groups=1),
        # tick 3, now 6: client entry (1, v3) (327-329); NextIndex 1 <= 1 ->
        # whole log, PrevLogIndex 0 (343-351); followers skip the checks
        # (LastApplied 0, 135), append, reply MatchIndex 1; histogram {1: 2}:
        # 4 > 3 and 1 > 0 -> CommitIndex 1 (381-391)
        stats(committed=1, ae_ok=2, leader_groups=1),
        # tick 4, now 8: entry (1, v4); NextIndex 2 <= 2 -> Logs [entry 2],
        # PrevLogIndex = MatchIndex 1, PrevLogTerm = GetLog(1).Term 1 (353-360);
        # checks pass, append; LeaderCommit 1 > 0 -> min(1, len+1 = 3) = 1
        # (151-152); histogram {2: 2} -> CommitIndex 2
        stats(committed=1, ae_ok=2, leader_groups=1),
    ]
    dc = draw_c(seed, gid, 0, 2)
    v3, v4 = client_value(seed, gid, 0, 3), client_value(seed, gid, 0, 4)
    log = [(1, v3), (1, v4)]
    final = [node(L, 1, 1, log, commit=2, deadline=4 + dc, timeout=dc, match=[0, 2, 2]),
             node(F, 1, 1, log, commit=1, deadline=8 + 20, timeout=20),   # reset by tick 4's AppendEntries
             node(F, 1, 1, log, commit=1, deadline=8 + 20, timeout=20)]
    return dict(cfg=cfg, R=R, start=[start], first_tick=0, per_tick=per_tick, final=[final], fault=[0])


def case_t2():
    seed, gid = 0x7E57_0002, 0
    R = 5
    a, b = 0x1111, 0x2222
    cfg = dict(replicas=R, groups=1, ring_depth=K, client_period=0, seed=seed)
    full = [(1, a), (2, b)]
    # S0 leads term 2 (MatchIndex: S1 2 -> NextIndex 3 > LastApplied 2, so S1
    # gets a heartbeat); S1 still leads the stale term 1 with the shorter log
    start = [node(L, 2, 1, full, commit=1, deadline=100, timeout=12, match=[0, 2, 2, 2, 2]),
             node(L, 1, 1, full[:1], commit=1, deadline=100, timeout=11, match=[1, 0, 1, 1, 1]),
             node(F, 2, 1, full, commit=1, deadline=100, timeout=21),
             node(F, 2, 1, full, commit=1, deadline=100, timeout=22),
             node(F, 2, 1, full, commit=1, deadline=100, timeout=23)]
    t = 10   # now 20
    d1 = draw_f(seed, gid, 1, t)   # S1's FollowerRun entry after stepping down (main.go:320 -> 114)
    per_tick = [
        # tick 10: S0's round. S1 (Leader): heartbeat PrevLogIndex 2, PrevLogTerm 2
        # (364-371); 2 > 1 -> Success with MatchIndex 0 (313-316), Follower, not
        # Voted, Term 2 (317-319). S2..S4: heartbeat, checks pass (137-146),
        # reset to 20 + d. MatchIndex {0, 2, 2, 2}: {2: 3} -> 6 > 5 and 2 > 1
        # -> CommitIndex 2. S1 is a Follower now: no round of its own.
        stats(committed=1, ae_ok=4, leader_groups=1),
        # tick 11: NextIndex[S1] = 1 <= 2 -> whole log, PrevLogIndex 0,
        # PrevLogTerm 2 (343-351). S1: timer reset first (124-127), 2 >= 2,
        # LastApplied 1 > 0, 1+2 < 0 false, GetLog(0) -> panic (142 -> 404):
        # the group freezes; S2..S4 get nothing this tick.
        stats(faults=1),
        zero_stats(),                 # tick 12: frozen
    ]
    final = [node(L, 2, 1, full, commit=2, deadline=100, timeout=12, match=[0, 0, 2, 2, 2]),
             node(F, 2, 0, full[:1], commit=1, deadline=22 + d1, timeout=d1),
             node(F, 2, 1, full, commit=1, deadline=20 + 21, timeout=21),
             node(F, 2, 1, full, commit=1, deadline=20 + 22, timeout=22),
             node(F, 2, 1, full, commit=1, deadline=20 + 23, timeout=23)]
    return dict(cfg=cfg, R=R, start=[start], first_tick=t, per_tick=per_tick, final=[final], fault=[1])


def case_t3():
    seed, gid = 0x7E57_0003, 0
    R = 3
    x, y = 0xAAAA, 0xBBBB
    cfg = dict(replicas=R, groups=1, ring_depth=K, client_period=0, seed=seed)
    log = [(1, x), (1, y)]
    start = [node(F, 1, 0, log, commit=1, deadline=2, timeout=20),
             node(F, 1, 0, log, commit=1, deadline=100, timeout=20),
             node(F, 1, 0, log, commit=1, deadline=100, timeout=22)]
    dc = draw_c(seed, gid, 0, 1)
    per_tick = [
        # tick 1, now 2: S0's timer fires (171-177): Term 2, Candidate; its round:
        # S1, S2 grant (2 >= 1, not Voted; Reset -> 2+20, 2+22); Leader with
        # MatchIndex 0 / NextIndex 1 (273-282)
        stats(elections_won=1, term_bumps=1, votes_granted=2, leader_groups=1),
        # tick 2, now 4: the new leader's first AppendEntries: NextIndex 1 <=
        # LastApplied 2 -> whole log, PrevLogIndex 0 (343-351). S1 resets its
        # timer (4+20), passes 129 and 137, then GetLog(0) panics (142 -> 404)
        stats(faults=1),
    ]
    final = [node(L, 2, 1, log, commit=1, deadline=2 + dc, timeout=dc, match=[0, 0, 0]),
             node(F, 2, 1, log, commit=1, deadline=4 + 20, timeout=20),
             node(F, 2, 1, log, commit=1, deadline=2 + 22, timeout=22)]
    return dict(cfg=cfg, R=R, start=[start], first_tick=1, per_tick=per_tick, final=[final], fault=[1])


def case_t4():
    seed = 0x7E57_0004
    R = 5
    cfg = dict(replicas=R, groups=1, ring_depth=K, client_period=0, seed=seed)
    start = [node(F, 3, 1, deadline=100, timeout=20),
             node(C, 3, 1, deadline=100, timeout=12),
             node(F, 2, 0, deadline=100, timeout=25),
             node(C, 3, 1, deadline=100, timeout=11),
             node(F, 1, 0, deadline=100, timeout=15)]
    t = 7   # now 14
    per_tick = [
        # S1's round (the first non-follower; rounds in ascending id). S0: Term 3
        # is not below 3 but S0 has Voted -> refuse, no reset (160-162). S2:
        # 3 >= 2, not Voted -> grant, Reset -> 14+25, Term 3, Voted (164-170).
        # S3 (Candidate, Term 3): 3 > 3 false -> the refusal goes into S3's OWN
        # VRes (242) and S3's timer is Reset -> 14+11 (243-246); S1 blocks at
        # 265 forever: fault, group frozen. S4 never gets the request.
        stats(votes_granted=1, faults=1),
        zero_stats(),                 # tick 8: frozen
    ]
    final = [node(F, 3, 1, deadline=100, timeout=20),
             node(C, 3, 1, deadline=100, timeout=12),
             node(F, 3, 1, deadline=14 + 25, timeout=25),
             node(C, 3, 1, deadline=14 + 11, timeout=11),
             node(F, 1, 0, deadline=100, timeout=15)]
    return dict(cfg=cfg, R=R, start=[start], first_tick=t, per_tick=per_tick, final=[final], fault=[2])


CASES = {"T1_election_first_entries_r3": case_t1, "T2_higher_term_leader_steps_down_r5": case_t2,
         "T3_new_leader_first_contact_panics_r3": case_t3, "T4_same_term_candidates_deadlock_r5": case_t4}

STAT_ORDER = ("committed", "elections_won", "term_bumps", "ae_ok", "ae_fail", "votes_granted", "faults",
              "leader_groups")


def run_case(make, name):
    """Load the case's start state into `make(**cfg)` (engine or oracle), tick
    one tick at a time, and check every per-tick stat and the final
    canonical view against the hand-derived values."""
    import numpy as np

    from harness import diff_states

    c = CASES[name]()
    x = make(**c["cfg"])
    x.load_state(build_state(c["start"], c["R"], K))
    for i, want in enumerate(c["per_tick"]):
        t = c["first_tick"] + i
        got = dict(zip(STAT_ORDER, [int(v) for v in x.tick(t, 1)]))
        assert got == want, f"{name}: stats of tick {t}: {got} != {want}"
    want = build_state(c["final"], c["R"], K, faults=c["fault"])
    got = x.store_state()
    # derived fields of the canonical view: REF NextIndex = MatchIndex + 1 for
    # a leader's peers (main.go:280-281, 376-377), high-water mark = LastApplied
    R = c["R"]
    for g in range(len(c["final"])):
        for r in range(R):
            want["hwm"][g, r] = want["last"][g, r]
            if want["role"][g, r] == L:
                for p in range(R):
                    if p != r:
                        want["next"][g, r, p] = want["match"][g, r, p] + 1
    d = diff_states(got, want)
    assert not d, f"{name}: final state differs from the hand-derived one:\n" + "\n".join(d)
    assert np.array_equal(got["fault"], np.array(c["fault"], np.uint8))
