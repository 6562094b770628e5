"""Diagnostics: run the comm / no-comm per-tick stats comparison of
test_side_stream_stats_sum_equals_host_sum several times under the current
environment and print which ticks differ (engine a vs b vs the oracle)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
from raftstep import Engine  # noqa: E402
import oracle  # noqa: E402

kw = dict(replicas=5, groups=3000, client_period=1, seed=0x5EED0003, isolate_per_65536=12000)
n = 40
o = oracle.Oracle(**kw)
o.init_new_nodes(0)
ro = np.array([o.tick(t, 1) for t in range(n)])
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for comm in (True, False):
        e = Engine(**kw)
        if comm:
            e.comm_init(1, 0, Engine.comm_unique_id())
        e.init_new_nodes(0)
        s = e.tick(0, n)
        r = e.tick_records(n)
        bad = [t for t in range(n) if list(r[t]) != list(ro[t])]
        print(f"rep {rep} comm {comm}: ticks differing from the oracle: {bad[:10]}",
              "" if not bad else f"first: engine {list(r[bad[0]])} oracle {list(ro[bad[0]])}", flush=True)
        e.close()
