"""GPU: BASELINE config C3 on the one GPU a box has — 16M (2^24) 5-replica
groups sharded as 8 engines of 2^21 groups (group_base = k * 2^21, the shards
8 ranks would own), against one 2^24-group engine and the CPU oracle.

Sharding is exact because Raft groups never address each other (the
reference's cluster is one `Nodes` map per group, main.go:12; every message
goes to a peer of the same group, main.go:259, 334) and the trace RNG is keyed
by the GLOBAL group id. So per shard and tick: the shard stats sum to the big
engine's, each shard's per-group digests equal the big engine's slice, their
wrapping sum equals its total, and a 700-group slice of every shard equals
the oracle started at that global offset. 48 ticks: past the wrap of the
K=32 ring."""
import numpy as np
import pytest

import oracle
from raftstep import Engine

pytestmark = pytest.mark.gpu

SHARD = 1 << 21
NSHARDS = 8
SLICE = 700
KW = dict(replicas=5, ring_depth=32, client_period=1, seed=0x5EED0003)


def test_c3_shards_equal_one_engine_and_the_oracle():
    big = Engine(groups=SHARD * NSHARDS, **KW)
    shards = [Engine(groups=SHARD, group_base=k * SHARD, **KW) for k in range(NSHARDS)]
    offs = [(k * 277_003) % (SHARD - SLICE) for k in range(NSHARDS)]
    slices = [oracle.Oracle(groups=SLICE, group_base=k * SHARD + offs[k], **KW) for k in range(NSHARDS)]
    for x in [big] + shards + slices:
        x.init_steady(0, 0)
    t = 1
    for k in (24, 24):
        sb = big.tick(t, k)
        ss = np.zeros(8, np.int64)
        for e in shards:
            ss += e.tick(t, k)
        assert list(ss) == list(sb), f"shard stats sum vs one engine, ticks [{t}, {t + k})"
        assert sb[0] == SHARD * NSHARDS * k and sb[6] == 0   # one commit per group and tick, no fault
        for o in slices:
            o.tick(t, k, threads=8)
        t += k
        dbig, tbig = big.state_digest()
        tot = 0
        for i, e in enumerate(shards):
            d, ts = e.state_digest()
            assert np.array_equal(d, dbig[i * SHARD:(i + 1) * SHARD]), f"shard {i} digests at tick {t - 1}"
            tot = (tot + ts) & 0xFFFFFFFFFFFFFFFF
            do, _ = slices[i].state_digest()
            assert np.array_equal(do, d[offs[i]:offs[i] + SLICE]), f"shard {i} oracle slice at tick {t - 1}"
        assert tot == tbig
    for x in [big] + shards + slices:
        x.close()
