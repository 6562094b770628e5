"""CPU checks of the audit tooling on the oracle: the state digest
(oracle_state_digest = raft_state_digest's definition) and trace
record/replay (raftstep.trace) — no GPU involved."""
import numpy as np
import pytest

import harness as H
import oracle
from raftstep import abi, trace


def test_digest_covers_every_canonical_field():
    rng = np.random.default_rng(5)
    G, R, K = 40, 3, 8
    st = H.random_state(rng, G, R, K)
    o = oracle.Oracle(replicas=R, groups=G, ring_depth=K)
    o.load_state(st)
    base, tot = o.state_digest()
    assert tot == int(base.sum(dtype=np.uint64))
    assert len(set(base.tolist())) == G
    for field, idx in [("term", (7, 1)), ("commit", (3, 0)), ("deadline", (9, 2)), ("timeout", (1, 1)),
                       ("voted", (2, 2)), ("fault", (5,))]:
        s2 = {k: v.copy() for k, v in st.items()}
        s2[field][idx] = s2[field][idx] + 1 if field != "voted" else 1 - s2[field][idx]
        o.load_state(s2)
        d, _ = o.state_digest()
        assert d[idx[0]] != base[idx[0]], field
        assert np.array_equal(np.delete(d, idx[0]), np.delete(base, idx[0])), field
    # a log entry inside the live window
    g, r = np.argwhere(st["last"] > 0)[0]
    s2 = {k: v.copy() for k, v in st.items()}
    s2["log_value"][g, r, (int(st["last"][g, r]) - 1) % K] ^= 1
    o.load_state(s2)
    assert o.state_digest()[0][g] != base[g]


def test_digest_is_shard_invariant():
    kw = dict(replicas=5, client_period=1, seed=0x5EED0004, isolate_per_65536=16384)
    whole = oracle.Oracle(groups=300, **kw)
    parts = [oracle.Oracle(groups=150, group_base=b, **kw) for b in (0, 150)]
    for x in [whole] + parts:
        x.init_new_nodes(0)
        x.tick(0, 60)
    dw, tw = whole.state_digest()
    d0, t0 = parts[0].state_digest()
    d1, t1 = parts[1].state_digest()
    assert np.array_equal(dw, np.concatenate([d0, d1]))
    assert tw == (t0 + t1) % 2**64


@pytest.mark.parametrize("sem", [abi.SEM_REF, abi.SEM_RAFT])
def test_trace_record_replay_on_oracle(tmp_path, sem):
    rng = np.random.default_rng(11 + sem)
    o = oracle.Oracle(replicas=5, groups=96, ring_depth=16, client_period=2, seed=77, semantics=sem,
                      isolate_per_65536=9000)
    rec = trace.TraceRecorder(o)
    rec.init_new_nodes(0)
    H.random_events(rec, rng, 30)
    path = tmp_path / "t.npz"
    rec.save(path)
    meta, arrays = trace.load(path)
    assert len(meta["events"]) == 30 and meta["config"]["semantics"] == sem
    trace.replay(path, oracle.Oracle)   # deterministic: replays clean


def test_trace_replay_reports_divergence(tmp_path):
    o = oracle.Oracle(replicas=3, groups=16, client_period=1, seed=5)
    rec = trace.TraceRecorder(o)
    rec.init_new_nodes(0)
    rec.tick(0, 40)
    rec.meta["config"]["seed"] = 6          # replay on a different trace seed
    rec.save(tmp_path / "t.npz")
    with pytest.raises(trace.Mismatch, match=r"(stats|digest)"):
        trace.replay(tmp_path / "t.npz", oracle.Oracle)
    # a digest-only divergence names the groups and dumps their nodelog lines
    o2 = oracle.Oracle(replicas=3, groups=16, client_period=1, seed=5)
    rec2 = trace.TraceRecorder(o2)
    rec2.init_new_nodes(0)
    rec2.tick(0, 40)
    rec2.meta["events"][0]["digest"] = "1"
    rec2.arrays["e0_gdig"] = rec2.arrays["e0_gdig"].copy()
    rec2.arrays["e0_gdig"][0] ^= np.uint64(1)
    rec2.save(tmp_path / "u.npz")
    with pytest.raises(trace.Mismatch, match=r"groups differ.*\n# group 0\n\[Server0:"):
        trace.replay(tmp_path / "u.npz", oracle.Oracle)


@pytest.mark.parametrize("name", ["trace_mixed_ref", "trace_mixed_raft", "trace_steady_crc"])
def test_golden_traces_replay_on_oracle(name):
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", f"{name}.npz")
    trace.replay(path, oracle.Oracle)
