"""GPU: the N>1 path through the ENGINE — two engine
processes on the one GPU, each owning a group_base shard of C3's form (the
steady split tick: two half launches on two streams, list skip), their
statistics summed across the processes with torch.distributed (gloo; two
RCCL ranks cannot share one device), compared with one engine over both
shards (per-group digests, summed stats) and with oracle slices, one of them
straddling the shard boundary. Groups never address each other (main.go:12,
259, 334) and the trace RNG is keyed by the global group id, so the shards
must reproduce the single engine exactly.

Also: the statistics all-reduce's timeout bounds the collective, not the
call: a long call under a single-rank communicator with a tiny
RAFTSTEP_COMM_TIMEOUT_S completes."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = (1 << 17) + 300                 # per rank (the split needs >= 2 x 65536)
KW = dict(replicas=5, ring_depth=32, client_period=1, seed=0x5EED0003)
CALLS = ((6, True), (20, True), (7, False), (20, True), (1, True))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(e):
    t, total = 1, np.zeros(8, np.int64)
    e.init_steady(0, 0)
    for k, st in CALLS:
        s = e.tick(t, k, stats=st)
        if st:
            total += s
        t += k
    e.sync()
    return total


def _worker(rank, world, port, outdir):
    sys.path[:0] = [os.path.join(ROOT, "raft-sample_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from raftstep import Engine
    from raftstep import dist as rdist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = Engine(groups=G, group_base=rank * G, **KW)
    e.diag_enable()
    local = _run(e)
    total = rdist.sum_over_ranks(dist, local)
    dig, _ = e.state_digest()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), local=local, total=np.array(total), digests=dig,
             skipped=e.diag_read()["ticks_list_skipped"])
    e.close()
    dist.barrier()
    dist.destroy_process_group()


def test_two_engine_processes_equal_one_engine_and_the_oracle(tmp_path):
    import torch.multiprocessing as mp

    import oracle
    from raftstep import Engine
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    one = Engine(groups=world * G, **KW)
    ref = _run(one)
    dig, _ = one.state_digest()
    got = np.concatenate([p["digests"] for p in parts])
    bad = np.nonzero(got != dig)[0]
    assert not bad.size, f"{bad.size} group digests differ between the shards and one engine, first {bad[:4]}"
    for p in parts:
        assert list(p["total"]) == list(ref)                    # the gloo sum of the shards' stats
        assert int(p["skipped"]) >= 40                          # each shard ran the steady split tick
    assert list(sum(p["local"] for p in parts)) == list(ref)
    assert ref[0] == world * G * sum(k for k, st in CALLS if st)
    # oracle slices: the first groups, across the shard boundary, the last groups
    for off in (0, G - 350, world * G - 700):
        o = oracle.Oracle(groups=700, group_base=off, **KW)
        o.init_steady(0, 0)
        t = 1
        for k, _ in CALLS:
            o.tick(t, k, threads=16)
            t += k
        do, _ = o.state_digest()
        assert (dig[off:off + 700] == do).all(), f"oracle slice at {off}"


def test_comm_timeout_bounds_the_collective_not_the_call(monkeypatch):
    """RAFTSTEP_COMM_TIMEOUT_S used to run from the moment
    raft_tick had queued the whole call, so a call whose compute outlasted it
    ended in RAFT_ETIMEDOUT with every rank present. Now the budget restarts
    at each all-reduce's marker: 300 churn ticks at 2^22 groups (~50 ms of
    compute, 8-tick windows of ~2 ms) under a 20-ms budget complete, stats
    equal to an engine without a communicator."""
    from raftstep import Engine
    kw = dict(replicas=7, groups=1 << 22, ring_depth=32, client_period=1, seed=0x5EED0004, semantics=1,
              isolate_per_65536=8192, isolate_leader=1)
    a, b = Engine(**kw), Engine(**kw)
    a.comm_init(1, 0, Engine.comm_unique_id())
    for e in (a, b):
        e.init_new_nodes(0)
        e.tick(0, 48)
    monkeypatch.setenv("RAFTSTEP_COMM_TIMEOUT_S", "0.02")
    import time
    t0 = time.perf_counter()
    sa = a.tick(48, 300)
    el = time.perf_counter() - t0
    sb = b.tick(48, 300)
    assert list(sa) == list(sb)
    assert el > 0.02, f"the call ({el * 1e3:.1f} ms) must outlast the budget for this test to mean anything"
    assert a.comm_info()[2] > 30        # one all-reduce per window
    print(f"300-tick call under a communicator: {el * 1e3:.1f} ms")
