"""CPU: EXT leader-isolation mode (isolate_leader = 1, SURVEY §8(d) C4:
"leader isolation ... for 8-32 ticks"). A window's victim is the lowest-id
Leader when the window's first tick begins; checked on the oracle against the
window schedule restated from the trace definition (kat_tick.trace_rng)."""
import numpy as np

import kat_tick
import oracle
from raftstep import abi

ST_ISOLATE = 4


def window(seed, gid, e, lo, hi):
    """(start, len) of epoch e's isolation window (every epoch has one at p = 65536)."""
    h = kat_tick.trace_rng(seed, gid, 0, ST_ISOLATE, e)
    return e * 32 + ((h >> 24) & 31), lo + ((h >> 32) % (hi - lo + 1))


def lowest_leader(st, g, R):
    ls = [r for r in range(R) if st["role"][g, r] == abi.LEADER]
    return ls[0] if ls else None


def test_victim_is_the_leader_at_the_window_start():
    R, G, seed = 5, 48, 0x1EAD
    kw = dict(replicas=R, groups=G, ring_depth=64, client_period=1, seed=seed, semantics=abi.SEM_RAFT,
              isolate_per_65536=65536, isolate_min_ticks=8, isolate_max_ticks=12, isolate_leader=1)
    o = oracle.Oracle(**kw)
    o.init_steady(0, 0)
    starts = {g: {e: window(seed, g, e, 8, 12)[0] for e in range(3)} for g in range(G)}
    seen = 0
    prev = o.store_state(logs=False)
    for t in range(1, 96):
        o.tick(t, 1)
        cur = o.store_state(logs=False)
        for g in range(G):
            for e, s in starts[g].items():
                if s != t:
                    continue
                # decided from the roles as the tick began = as the previous tick ended
                L = lowest_leader(prev, g, R)
                nib = (int(cur["iso_victim"][g]) >> (4 * (e & 1))) & 0xF
                assert nib == (8 | L if L is not None else 0), (g, e, t, nib, L)
                seen += 1
        prev = cur
    assert seen == sum(1 <= s <= 95 for g in range(G) for s in starts[g].values()) > 2 * G


def test_isolated_leader_is_cut_off_and_the_rest_elect():
    """While the victim (the leader) is cut off, its AppendEntries are dropped
    (counted as failures) and, once the followers' timers expire, the others
    elect a second leader; the hashed mode of the same trace isolates a
    hashed replica instead, so the two traces differ."""
    R, G, seed = 5, 64, 0x1EAE
    base = dict(replicas=R, groups=G, ring_depth=64, client_period=1, seed=seed, semantics=abi.SEM_RAFT,
                isolate_per_65536=65536, isolate_min_ticks=30, isolate_max_ticks=32)
    lead = oracle.Oracle(isolate_leader=1, **base)
    hashed = oracle.Oracle(**base)
    for x in (lead, hashed):
        x.init_steady(0, 0)
    a, b = lead.tick(1, 60), hashed.tick(1, 60)
    assert a[abi.STAT_NAMES.index("elections_won")] > 0 and list(a) != list(b)
    st = lead.store_state(logs=False)
    assert (st["iso_victim"] != 0).mean() > 0.5   # (a window that began leaderless, or at tick 0, has none)
