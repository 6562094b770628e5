"""Diagnostic: per-launch fast-kernel time (profile mode 1) early and late in
a run, for C4 and simplified variants, to locate what slows the steady-state
kernel under churn."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-sample_amd"))
from raftstep import Engine  # noqa: E402

G = int(os.environ.get("PROBE_GROUPS", 1 << 22))
VARIANTS = {
    "c4": dict(replicas=7, semantics=1, ring_depth=128, isolate_per_65536=8192, isolate_min_ticks=8,
               isolate_max_ticks=32, init="new"),
    "c4_noiso": dict(replicas=7, semantics=1, ring_depth=128, init="new"),
    "r7_raft_steady": dict(replicas=7, semantics=1, ring_depth=128, init="steady"),
    "r7_ref_steady": dict(replicas=7, semantics=0, ring_depth=128, init="steady"),
    "r7_ref_steady_k32": dict(replicas=7, semantics=0, ring_depth=32, init="steady"),
    "r7_raft_steady_hashed_leader": dict(replicas=7, semantics=1, ring_depth=128, init="steady-1"),
    "r7_raft_steady_iso": dict(replicas=7, semantics=1, ring_depth=128, isolate_per_65536=8192,
                               isolate_min_ticks=8, isolate_max_ticks=32, init="steady"),
}
names = sys.argv[1:] or list(VARIANTS)
for name in names:
    kw = dict(VARIANTS[name])
    init = kw.pop("init")
    e = Engine(groups=G, client_period=1, entries_per_tick=1, seed=0x5EED0002, **kw)
    if init == "new":
        e.init_new_nodes(0)
        t = 48
        e.tick(0, 48, stats=False)
    else:
        e.init_steady(-1 if init == "steady-1" else 0, 0)
        t = 1
    out = []
    for rep in range(6):
        e.profile(1)
        e.tick(t, 16, stats=False)
        ms, n = e.profile_read()
        e.profile(0)
        e.profile(2)
        e.tick(t + 16, 16, stats=True)
        ms2, n2 = e.profile_read()
        e.profile(0)
        out.append((t, round(ms / n * 1e3, 1), round(ms2 / n2 * 1e3, 1)))
        t += 32
    print(name, "(tick, fast-kernel us, region us/tick):", out, flush=True)
    e.close()
