"""Diagnostics: per-tick lane-class counts of a bench workload at full size
in its timed region (after settle + warm-up), from raft_diag_read."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "raft-sample_amd")):
    sys.path.insert(0, p)
import bench  # noqa: E402
from raftstep import Engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
wl = bench.WORKLOADS[name]
R = wl.get("replicas", 5)
kw = bench.engine_kwargs(wl, R, wl["groups"], 0, wl["ring_depth"], wl["entries"], wl["crc"])
e = Engine(**kw)
if wl.get("init") == "new":
    e.init_new_nodes(0)
    e.tick(0, wl["settle"])
    t = wl["settle"]
else:
    e.init_steady(0, 0)
    t = 1
e.tick(t, 25)
t += 25
e.diag_enable()
n = 40
s = e.tick(t, n)
c = e.diag_read()
print("stats per tick", [round(x / n) for x in s.tolist()])
for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v / n:12.0f} per tick")
