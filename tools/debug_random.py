"""Diagnostic: test_gpu_raft.test_raft_random_state_ticks's setup (argument
R) or one of its TRACES (argument: the trace name), ticked in the test's own
chunks (or STEP ticks at a time), printing the groups whose canonical state
differs from the oracle first, field by field.

    python tools/debug_random.py R|TRACE_NAME
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import test_gpu_raft as TR  # noqa: E402


def main():
    arg = sys.argv[1]
    if arg.isdigit():
        R = int(arg)
        step = int(os.environ.get("STEP", "3"))
        rng = np.random.default_rng(9100 + R)
        G, K = 300, 16
        e, o = TR.pair(replicas=R, groups=G, ring_depth=K, seed=0x7E + R, client_period=1,
                       isolate_per_65536=12000, isolate_min_ticks=2, isolate_max_ticks=16)
        st = TR.random_raft_state(rng, G, R, K)
        e.load_state(st)
        o.load_state(st)
        t0, n = 30, 60
    else:
        kw, init, t0, n, every = TR.TRACES[arg]
        step = int(os.environ.get("STEP", str(every)))
        G = kw["groups"]
        e, o = TR.pair(**kw)
        for x in (e, o):
            if init == "new":
                x.init_new_nodes(t0)
            else:
                x.init_steady(-1 if init == "steady-1" else 0, t0 - 1 if t0 else 0)
    pe = e.store_state()
    for t in range(t0, t0 + n, step):
        a, b = e.tick(t, step), o.tick(t, step)
        x, y = e.store_state(), o.store_state()
        bad = set()
        for k in x:
            d = np.asarray(x[k]) != np.asarray(y[k])
            if d.any():
                bad |= set(np.nonzero(d.reshape(G, -1).any(axis=1))[0].tolist())
        if bad or list(a) != list(b):
            print(f"ticks {t}..{t + step - 1}: stats engine {list(a)} oracle {list(b)}; groups {sorted(bad)[:10]}")
            for g in sorted(bad)[:2]:
                for k in x:
                    if k.startswith("log"):
                        continue
                    print(f"  g{g} {k:10s} before {np.asarray(pe[k])[g].reshape(-1).tolist()}")
                    print(f"  g{g} {k:10s} engine {np.asarray(x[k])[g].reshape(-1).tolist()}")
                    print(f"  g{g} {k:10s} oracle {np.asarray(y[k])[g].reshape(-1).tolist()}")
                for k in ("log_term",):
                    print(f"  g{g} {k} before {np.asarray(pe[k])[g].reshape(-1).tolist()}")
                    print(f"  g{g} {k} engine {np.asarray(x[k])[g].reshape(-1).tolist()}")
                    print(f"  g{g} {k} oracle {np.asarray(y[k])[g].reshape(-1).tolist()}")
            return 1
        pe = x
    print("no difference")
    return 0


if __name__ == "__main__":
    sys.exit(main())
