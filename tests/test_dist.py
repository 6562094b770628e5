"""CPU multi-process (gloo, world_size 2) checks of the sharded path:
group sharding by id is invariant (per-group state and summed stats equal a
single-process run) and the rank-0 id exchange / max-over-ranks timing
helpers behave. The CPU oracle stands in for the GPU engine here; the RCCL
sum itself runs on the GPU box (tests/test_gpu_dist.py)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = dict(replicas=5, client_period=1, seed=0x5EED0003, isolate_per_65536=12000, isolate_min_ticks=4,
           isolate_max_ticks=24)
G_TOTAL, TICKS = 301, 90


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    sys.path[:0] = [os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import harness
    import oracle
    from raftstep import dist as rdist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base, n = rdist.shard(G_TOTAL, world, rank)
    o = oracle.Oracle(groups=n, group_base=base, **CFG)
    o.init_new_nodes(0)
    stats = o.tick(0, TICKS)
    total = rdist.sum_over_ranks(dist, stats)
    uid = rdist.exchange_comm_id(dist, rank, lambda: b"\x07" * 128)
    slowest = rdist.max_over_ranks(dist, 1.5 + rank)
    h = harness.group_hashes(o.store_state())
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), base=base, n=n, total=np.array(total), hashes=h,
             uid=np.frombuffer(uid, np.uint8), slowest=slowest)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_equals_single_process(tmp_path, oracle_mod):
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    import harness
    o = oracle_mod.Oracle(groups=G_TOTAL, **CFG)
    o.init_new_nodes(0)
    ref_stats = o.tick(0, TICKS)
    ref_h = harness.group_hashes(o.store_state())
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    got = np.concatenate([p["hashes"] for p in parts])
    assert sum(int(p["n"]) for p in parts) == G_TOTAL
    assert (got == ref_h).all()
    for p in parts:
        assert list(p["total"]) == list(ref_stats)
        assert bytes(p["uid"]) == b"\x07" * 128
        assert float(p["slowest"]) == 2.5
    assert ref_stats[1] > 0  # elections happened


def test_shard_rejects_empty_shards():
    """groups_total < world would leave a rank with 0 groups, which
    raft_engine_create rejects: shard() says so up front."""
    from raftstep import dist as rdist
    with pytest.raises(ValueError, match="cannot be sharded"):
        rdist.shard(5, 8, 0)


@pytest.mark.parametrize("total,world", [(10, 3), (1 << 20, 8), (7, 7), (1 << 24, 8)])
def test_shard_ranges_cover_exactly(total, world):
    from raftstep import dist as rdist
    spans = [rdist.shard(total, world, r) for r in range(world)]
    assert spans[0][0] == 0
    for (b0, n0), (b1, _) in zip(spans, spans[1:]):
        assert b0 + n0 == b1
    assert sum(n for _, n in spans) == total
