"""Diagnostics: replay the block of W groups around group g with the bench
call structure up to tick T0, then one tick per call, comparing the whole
state with the oracle after every tick; on the first difference print the
group's state before/after on both sides and the engine's raw group words."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import oracle  # noqa: E402
from raftstep import Engine, abi  # noqa: E402

name, g, W, T0, T1 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
wl = bench.WORKLOADS[name]
R = wl.get("replicas", 5)
base = g - g % W
x = g - base
kw = bench.engine_kwargs(wl, R, W, base, wl["ring_depth"], wl["entries"], wl["crc"])
e, o = Engine(**kw), oracle.Oracle(**kw)
e.init_new_nodes(0)
o.init_new_nodes(0)
t = 0
for k in [wl["settle"], 5] + [20] * 15:
    k = min(k, T0 - t)
    if k <= 0:
        break
    e.tick(t, k)
    o.tick(t, k)
    t += k


def view(st):
    return {k: st[k][x].tolist() for k in abi.STATE_FIELDS if not k.startswith("log")}


def logs(st):
    K = st["log_term"].shape[-1]
    return {r: [(int(st["log_term"][x, r, (i - 1) % K])) for i in range(max(1, st["last"][x, r] - 12), st["last"][x, r] + 1)]
            for r in range(R)}


prev_e, prev_o = e.store_state(), o.store_state()
print("start at", t, "words", e.debug_group_words(x))
while t < T1:
    w0 = e.debug_group_words(x)
    se, so = e.tick(t, 1), o.tick(t, 1)
    try:
        a = e.store_state()
    except Exception as ex:
        print(f"tick {t}: store failed: {ex}")
        print("words before", w0, "\nwords after", e.debug_group_words(x))
        print("before engine", view(prev_e), "\nlogs", logs(prev_e))
        print("oracle after", view(o.store_state()), "\nlogs", logs(o.store_state()))
        break
    b = o.store_state()
    diff = [k for k in abi.STATE_FIELDS if not np.array_equal(a[k][x], b[k][x])]
    if diff:
        print(f"tick {t}: fields {diff}")
        print("words before", w0, "\nwords after", e.debug_group_words(x))
        for tag, st in (("before engine", prev_e), ("before oracle", prev_o), ("after engine", a), ("after oracle", b)):
            print(tag, view(st), "\n  logs(last 13)", logs(st))
        break
    prev_e, prev_o = a, b
    t += 1
else:
    print("no difference up to", T1)
