"""Replays a committed golden trace (tests/golden/*.npz) through an
implementation (oracle or engine) and compares per-group state digests every
few ticks, the per-interval stats and the final state."""
import os

import numpy as np

import harness

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["c1_r3_newnode", "c4_r7_iso", "c2_r5_steady", "c5_r5_e64"]


def spec(name):
    import importlib.util
    s = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "make_golden.py"))
    m = importlib.util.module_from_spec(s)
    s.loader.exec_module(m)
    return m.TRACES[name]


def check(make, name):
    sp = spec(name)
    gold = np.load(os.path.join(HERE, f"{name}.npz"), allow_pickle=False)
    impl = make(sp["cfg"])
    if sp["init"] == "new":
        impl.init_new_nodes(0)
    else:
        impl.init_steady(-1 if sp["init"] == "steady-1" else 0, 0)
    t0 = int(gold["t0"])
    t, i = t0, 0
    while t < t0 + sp["ticks"]:
        k = min(sp["every"], t0 + sp["ticks"] - t)
        s = impl.tick(t, k)
        t += k
        assert list(s) == list(gold["stats"][i]), f"{name}: stats differ at interval {i}"
        h = harness.group_hashes(impl.store_state())
        bad = np.nonzero(h != gold["hashes"][i])[0]
        assert bad.size == 0, f"{name}: groups {bad[:8].tolist()} differ after tick {t - 1}"
        i += 1
    final = impl.store_state()
    ref = {k[len("final_"):]: gold[k] for k in gold.files if k.startswith("final_")}
    harness.assert_same_state(final, ref, name)
