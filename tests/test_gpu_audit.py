"""GPU: the audit surface of the C-ABI — raft_state_digest (device) against
oracle_state_digest, including full-size (2^20-group) parity of the C2 and C4
shapes through the digest; raft_nodelog against the oracle's nodelog lines;
checkpoint save/load round trips; trace record on the engine / replay on the
oracle and replay of the committed oracle-recorded golden traces."""
import os

import numpy as np
import pytest

import harness as H
import oracle
from raftstep import Engine, RaftError, abi, checkpoint, trace

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
THREADS = min(16, os.cpu_count() or 1)


def both(**kw):
    return Engine(**kw), oracle.Oracle(**kw)


def assert_same_digest(e, o, what):
    de, te = e.state_digest()
    do, to = o.state_digest()
    bad = np.nonzero(de != do)[0]
    if bad.size:
        g = int(bad[0])
        raise AssertionError(f"{what}: {bad.size} group digests differ, first {bad[:8].tolist()}\n"
                             f"engine:\n{e.nodelog(g)}oracle:\n{o.nodelog(g)}")
    assert te == to, what


DIGEST_CASES = {
    "ref_newnode_r3": (dict(replicas=3, groups=700, client_period=3, seed=0x5EED0001, isolate_per_65536=8000),
                       "new", 0, 160),
    "ref_steady_msync_r5": (dict(replicas=5, groups=2000, client_period=1, ring_depth=16, seed=0x5EED0002), "steady",
                            1, 40),
    "raft_churn_r7": (dict(replicas=7, groups=1024, client_period=1, ring_depth=64, semantics=abi.SEM_RAFT,
                           seed=0x44, isolate_per_65536=20000, isolate_min_ticks=4, isolate_max_ticks=32),
                      "new", 0, 200),
    "raft_leader_iso_r7": (dict(replicas=7, groups=1024, client_period=1, ring_depth=64, semantics=abi.SEM_RAFT,
                                seed=0x45, isolate_per_65536=20000, isolate_min_ticks=4, isolate_max_ticks=32,
                                isolate_leader=1), "new", 0, 200),
    # small ring, frequent leader-isolation windows, long run: elections, stale
    # leaders, returns and truncations in the fast path, ring phase segments
    # switching again while the previous segment is still live (three segments)
    "raft_leader_iso_k16_long": (dict(replicas=5, groups=2048, client_period=1, ring_depth=16, semantics=abi.SEM_RAFT,
                                      seed=0x46, isolate_per_65536=30000, isolate_min_ticks=4, isolate_max_ticks=16,
                                      isolate_leader=1), "new", 0, 600),
    "raft_hashed_iso_k32_long": (dict(replicas=7, groups=1024, client_period=1, ring_depth=32, semantics=abi.SEM_RAFT,
                                      seed=0x47, isolate_per_65536=30000, isolate_min_ticks=4, isolate_max_ticks=24),
                                 "new", 0, 500),
    "crc_e16_r5": (dict(replicas=5, groups=512, client_period=1, entries_per_tick=16, ring_depth=64, payload_crc=1,
                        corrupt_per_65536=3000, seed=0x5EED0005), "steady", 1, 20),
}


@pytest.mark.parametrize("name", sorted(DIGEST_CASES))
def test_device_digest_matches_oracle(name):
    kw, init, t0, n = DIGEST_CASES[name]
    e, o = both(**kw)
    for x in (e, o):
        x.init_new_nodes(0) if init == "new" else x.init_steady(-1, 0)
    assert_same_digest(e, o, f"{name}: init")
    t = t0
    while t < t0 + n:
        k = min(10, t0 + n - t)
        assert list(e.tick(t, k)) == list(o.tick(t, k, threads=THREADS)), f"{name}: stats at {t}"
        assert_same_digest(e, o, f"{name}: after tick {t + k - 1}")
        t += k
    # the digest is a function of the canonical view: equal to the digest of a
    # fresh engine loaded with that view
    st = e.store_state()
    e2 = Engine(**kw)
    e2.load_state(st)
    assert e2.state_digest()[1] == e.state_digest()[1]


def test_full_size_c2_digest_parity():
    """BASELINE config C2 at full size: 2^20 groups x R=5, K=32, steady state,
    every group's state equal to the oracle's (through the per-group digest;
    the whole canonical view would be ~1 GB) after 24 ticks and again after
    48, past the wrap of the 32-slot ring."""
    kw = dict(replicas=5, groups=1 << 20, ring_depth=32, client_period=1, seed=0x5EED0002)
    e, o = both(**kw)
    e.init_steady(0, 0)
    o.init_steady(0, 0)
    for t, k in ((1, 24), (25, 24)):
        se = e.tick(t, k)
        so = o.tick(t, k, threads=THREADS)
        assert list(se) == list(so)
        assert_same_digest(e, o, f"C2 full size after tick {t + k - 1}")


def test_full_size_c4_shape_digest_parity():
    """BASELINE config C4's shape (R=7, NewNode start, isolation churn, RAFT
    semantics) on 2^20 groups through the per-group digest."""
    kw = dict(replicas=7, groups=1 << 20, ring_depth=128, client_period=1, seed=0x5EED0002,
              semantics=abi.SEM_RAFT, isolate_per_65536=8192, isolate_min_ticks=8, isolate_max_ticks=32)
    e, o = both(**kw)
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    for t, k in ((0, 48), (48, 16)):
        assert list(e.tick(t, k)) == list(o.tick(t, k, threads=THREADS)), f"stats [{t}, {t + k})"
    assert_same_digest(e, o, "C4 shape full size after 64 ticks")


def test_full_size_c4_shape_digest_parity_past_ring_wrap():
    """C4's shape (R=7, NewNode start, isolation churn, RAFT) on 2^20 groups
    with K=64 for 160 ticks: past the wrap of the 2K = 128 physical ring slots
    (KP = 2K under isolation churn), so ring phase-segment switches and slot
    reuse happen at full size; digest parity at three points."""
    kw = dict(replicas=7, groups=1 << 20, ring_depth=64, client_period=1, seed=0x5EED0004,
              semantics=abi.SEM_RAFT, isolate_per_65536=8192, isolate_min_ticks=8, isolate_max_ticks=32)
    e, o = both(**kw)
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    for k in (48, 56, 56):
        assert list(e.tick(t, k)) == list(o.tick(t, k, threads=THREADS)), f"stats [{t}, {t + k})"
        t += k
        assert_same_digest(e, o, f"C4 shape K=64 full size after tick {t - 1}")


def test_nodelog_matches_oracle():
    kw = dict(replicas=3, groups=64, client_period=2, seed=0x5EED0001)
    e, o = both(**kw)
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    e.tick(0, 50)
    o.tick(0, 50)
    for g in range(0, 64, 7):
        assert e.nodelog(g) == o.nodelog(g)
    line = e.nodelog(0).splitlines()[0]
    assert line.startswith("[Server0:") and line.endswith(("][follower]", "][candidate]", "][leader]"))
    with pytest.raises(RaftError):
        e.nodelog(64)


@pytest.mark.parametrize("sem,crc", [(abi.SEM_REF, 0), (abi.SEM_RAFT, 0), (abi.SEM_REF, 1)])
def test_checkpoint_round_trip(tmp_path, sem, crc):
    kw = dict(replicas=5, groups=777, ring_depth=32, client_period=1, seed=0xC0DE, semantics=sem, payload_crc=crc,
              isolate_per_65536=12000, entries_per_tick=2)
    a = Engine(**kw)
    a.init_new_nodes(0)
    a.tick(0, 60)
    path = tmp_path / "ck.bin"
    a.save_checkpoint(path)
    b = Engine(**kw)
    b.load_checkpoint(path)
    assert b.state_digest()[1] == a.state_digest()[1]
    # continuing from the checkpoint is the same as never stopping
    assert list(a.tick(60, 40)) == list(b.tick(60, 40))
    assert b.state_digest()[1] == a.state_digest()[1]
    # the file is the canonical view: loaded into the oracle it continues identically
    cfg, st = checkpoint.read(path)
    assert cfg.groups == 777 and cfg.semantics == sem
    o = oracle.Oracle(**kw)
    o.load_state(st)
    c = Engine(**kw)
    c.load_checkpoint(path)
    assert o.state_digest()[1] == c.state_digest()[1]
    assert list(o.tick(60, 20)) == list(c.tick(60, 20))
    assert o.state_digest()[1] == c.state_digest()[1]


def test_checkpoint_rejects_corruption_and_mismatch(tmp_path):
    kw = dict(replicas=3, groups=100, seed=1)
    a = Engine(**kw)
    a.init_new_nodes(0)
    path = tmp_path / "ck.bin"
    a.save_checkpoint(path)
    data = bytearray(path.read_bytes())
    data[len(data) // 2] ^= 0x10
    bad = tmp_path / "bad.bin"
    bad.write_bytes(bytes(data))
    with pytest.raises(RaftError, match="CRC32C"):
        Engine(**kw).load_checkpoint(bad)
    with pytest.raises(RaftError, match="does not fit"):
        Engine(replicas=5, groups=100, seed=1).load_checkpoint(path)
    with pytest.raises(RaftError, match="truncated|CRC32C"):
        short = tmp_path / "short.bin"
        short.write_bytes(bytes(data[:400]))
        Engine(**kw).load_checkpoint(short)
    # the Python reader verifies the trailer too
    with pytest.raises(ValueError, match="CRC32C"):
        checkpoint.read(bad)
    # another shard's or another trace's checkpoint would resume on a different RNG stream
    with pytest.raises(RaftError, match="group_base"):
        Engine(**dict(kw, group_base=100)).load_checkpoint(path)
    with pytest.raises(RaftError, match="seed"):
        Engine(**dict(kw, seed=2)).load_checkpoint(path)
    with pytest.raises(RaftError, match="client_period"):
        Engine(**dict(kw, client_period=1)).load_checkpoint(path)
    # saving goes through <path>.tmp + rename: no temporary is left behind
    a.save_checkpoint(path)
    assert not (tmp_path / "ck.bin.tmp").exists()
    assert Engine(**kw).load_checkpoint(path) is None


@pytest.mark.parametrize("sem", [abi.SEM_REF, abi.SEM_RAFT])
def test_trace_recorded_on_engine_replays_on_oracle(tmp_path, sem):
    rng = np.random.default_rng(40 + sem)
    kw = dict(replicas=5, groups=300, ring_depth=16, client_period=1, seed=0x7ACE, semantics=sem,
              isolate_per_65536=10000)
    rec = trace.TraceRecorder(Engine(**kw))
    rec.init_new_nodes(0)
    H.random_events(rec, rng, 40, t0=1)
    rec.save(tmp_path / "t.npz")
    trace.replay(tmp_path / "t.npz", oracle.Oracle)
    trace.replay(tmp_path / "t.npz", Engine)


@pytest.mark.parametrize("name", ["trace_mixed_ref", "trace_mixed_raft", "trace_steady_crc"])
def test_golden_traces_replay_on_engine(name):
    trace.replay(os.path.join(GOLDEN, f"{name}.npz"), Engine)
