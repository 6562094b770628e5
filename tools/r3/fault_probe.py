"""Diagnostics: run a bench workload with per-call stats, find faulted
groups and replay a few of them on the oracle (group_base = the group)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import oracle  # noqa: E402
from raftstep import Engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
G = int(sys.argv[2]) if len(sys.argv) > 2 else None
wl = bench.WORKLOADS[name]
R = wl.get("replicas", 5)
G = G or wl["groups"]
kw = bench.engine_kwargs(wl, R, G, 0, wl["ring_depth"], wl["entries"], wl["crc"])
e = Engine(**kw)
e.diag_enable()
e.init_new_nodes(0)
t = 0
for k in [wl["settle"], 5] + [20] * 15:
    s = e.tick(t, k)
    rec = e.tick_records(k)
    f = rec[:, 6]
    print(f"ticks [{t},{t + k}) stats {s.tolist()} faults/tick {f.nonzero()[0].tolist()[:10]}", flush=True)
    t += k
print("classes", e.diag_read(), flush=True)
faulted = []
for g0 in range(0, G, 1 << 20):
    n = min(1 << 20, G - g0)
    st = e.store_state_range(g0, n, logs=False)
    idx = np.nonzero(st["fault"])[0]
    faulted += [(g0 + int(i), int(st["fault"][i])) for i in idx]
print("faulted groups", len(faulted), faulted[:20], flush=True)
codes = {}
for _, c in faulted:
    codes[c] = codes.get(c, 0) + 1
print("fault codes", codes, flush=True)
for g, c in faulted[:4]:
    o = oracle.Oracle(**dict(kw, groups=1, group_base=g))
    o.init_new_nodes(0)
    tt = 0
    for k in [wl["settle"], 5] + [20] * 15:
        o.tick(tt, k)
        tt += k
    so = o.store_state(logs=False)
    print(f"group {g}: engine fault {c}, oracle fault {int(so['fault'][0])}", flush=True)
    print("engine:\n" + e.nodelog(g) + "oracle:\n" + o.nodelog(0), flush=True)
