"""Diagnostics: re-run the block of W groups around group g of a bench
workload (group_base = g rounded down to W, so wave neighbours and ring
tiles are the same as in the full-size run) with the bench's call
structure against the oracle; print the first call whose state differs and
the differing fields. With STEP=1 the failing call is then replayed one
tick per call from a fresh start."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import harness as H  # noqa: E402
import oracle  # noqa: E402
from raftstep import Engine, abi  # noqa: E402

name, g = sys.argv[1], int(sys.argv[2])
W = int(sys.argv[3]) if len(sys.argv) > 3 else 256
wl = bench.WORKLOADS[name]
R = wl.get("replicas", 5)
kw = bench.engine_kwargs(wl, R, W, g - g % W, wl["ring_depth"], wl["entries"], wl["crc"])
calls = [wl["settle"], 5] + [20] * 15


def run(calls, stop_on_diff=True, verbose=True):
    e, o = Engine(**kw), oracle.Oracle(**kw)
    e.init_new_nodes(0)
    o.init_new_nodes(0)
    t = 0
    prev = None
    for k in calls:
        se, so = e.tick(t, k), o.tick(t, k)
        a, b = e.store_state(), o.store_state()
        bad = sorted({int(i) for kf in a for i in np.nonzero((a[kf] != b[kf]).reshape(W, -1).any(axis=1))[0]})
        if bad or list(se) != list(so):
            print(f"call [{t}, {t + k}): groups differ (local) {bad[:10]}; stats engine {se.tolist()} oracle {so.tolist()}")
            for x in bad[:2]:
                print(f"group {kw['group_base'] + x}:")
                for kf in abi.STATE_FIELDS:
                    if not np.array_equal(a[kf][x], b[kf][x]):
                        print(f"  {kf}: engine {a[kf][x].tolist()}\n  {' ' * len(kf)}  oracle {b[kf][x].tolist()}")
                        if prev is not None:
                            print(f"  {' ' * len(kf)}  before {prev[kf][x].tolist()}")
                print("engine:\n" + e.nodelog(x) + "oracle:\n" + o.nodelog(x))
            return t, k, bad
        prev = b
        t += k
    print("no difference")
    return None


r = run(calls)
if r and os.environ.get("STEP"):
    t0, k, bad = r
    # replay: the same calls up to t0, then one tick per call
    pre, s = [], 0
    for k2 in calls:
        if s >= t0:
            break
        pre.append(k2)
        s += k2
    print("--- replay one tick per call from", t0)
    run(pre + [1] * k)
