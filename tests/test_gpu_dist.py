"""GPU: the engine's RCCL statistics path with a single-rank communicator
(the box has one GPU; the 8-GPU run is the driver's scaling bench)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_single_rank_stats():
    from raftstep import Engine
    kw = dict(replicas=5, groups=5000, client_period=1, seed=0x5EED0003)
    a = Engine(**kw)
    b = Engine(**kw)
    a.comm_init(1, 0, Engine.comm_unique_id())
    for e in (a, b):
        e.init_steady(0, 0)
    sa, sb = a.tick(1, 10), b.tick(1, 10)
    assert list(sa) == list(sb) == [50000, 0, 0, 200000, 0, 0, 0, 50000]
    assert list(a.allreduce_stats(sa)) == list(sa)


def test_group_base_shards_are_invariant():
    """Two engines owning halves of the id space reproduce one engine."""
    from raftstep import Engine
    import harness
    kw = dict(replicas=5, client_period=1, seed=0x5EED0003, isolate_per_65536=12000)
    full = Engine(groups=1000, **kw)
    lo = Engine(groups=400, group_base=0, **kw)
    hi = Engine(groups=600, group_base=400, **kw)
    tot = np.zeros(8, np.int64)
    for e in (full, lo, hi):
        e.init_new_nodes(0)
    ref = full.tick(0, 80)
    tot += lo.tick(0, 80)
    tot += hi.tick(0, 80)
    assert list(tot) == list(ref)
    f = full.store_state()
    parts = [lo.store_state(), hi.store_state()]
    joined = {k: np.concatenate([p[k] for p in parts]) for k in f}
    harness.assert_same_state(joined, f, "sharded")
