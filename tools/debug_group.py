"""Diagnostic: replay one group of a full-size run alone (the trace is keyed
by the global group id, so an engine of 1 group at group_base=g reproduces
it), tick by tick against the oracle, and print the first tick whose
canonical state differs with every field of both sides before and after.

    python tools/debug_group.py GROUP TICKS '<json engine kwargs>'
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from raftstep import Engine  # noqa: E402


def show(tag, st):
    print(tag)
    for k, v in st.items():
        if k.startswith("log"):
            continue
        print("  %-10s %s" % (k, np.asarray(v).reshape(-1).tolist()))


def main():
    g, n = int(sys.argv[1]), int(sys.argv[2])
    kw = json.loads(sys.argv[3])
    kw.update(groups=1, group_base=g)
    e, o = Engine(**kw), oracle.Oracle(**kw)
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    pe, po = e.store_state(), o.store_state()
    for t in range(n):
        se, so = e.tick(t, 1), o.tick(t, 1)
        a, b = e.store_state(), o.store_state()
        diff = [k for k in a if not np.array_equal(a[k], b[k])]
        if diff or list(se) != list(so):
            print(f"tick {t}: fields {diff}; stats engine {list(se)} oracle {list(so)}")
            show("before (engine):", pe)
            show("before (oracle):", po)
            show("after (engine):", a)
            show("after (oracle):", b)
            for k in diff:
                if k.startswith("log"):
                    print(k, "engine", np.asarray(a[k]).reshape(-1).tolist()[:64])
                    print(k, "oracle", np.asarray(b[k]).reshape(-1).tolist()[:64])
            return 1
        pe, po = a, b
    print("no difference in", n, "ticks")
    return 0


if __name__ == "__main__":
    sys.exit(main())
