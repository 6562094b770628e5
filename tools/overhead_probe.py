"""Per-call host overhead of raft_tick on a C2 engine (median wall time of
single calls): torch.cuda.synchronize, ticks of 1 / 2 / 20 with and without
statistics, the split steady tick on / off (RAFTSTEP_SPLIT_STEADY)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raft-sample_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from raftstep import Engine  # noqa: E402


def tm(f, n=100):
    f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[n // 2] * 1e6, 1)


torch.cuda.init()
torch.cuda.synchronize()
print("torch.cuda.synchronize us", tm(torch.cuda.synchronize))
wl = bench.WORKLOADS["C2"]
for split in ("1", "0"):
    os.environ["RAFTSTEP_SPLIT_STEADY"] = split
    e = Engine(**bench.engine_kwargs(wl, 5, 1 << 20, 0, 32, 1, 0))
    e.init_steady(0, 0)
    e.tick(1, 6)
    t = [7]

    def tk(k, st=True, dev_sync=False):
        def f():
            e.tick(t[0], k, stats=st)
            if not st:
                e.sync()
            if dev_sync:   # (bench.py's timed region ends with torch.cuda.synchronize)
                torch.cuda.synchronize()
            t[0] += k
        return f
    r = {f"tick{k}{'' if st else '_nostats'}": tm(tk(k, st)) for k in (1, 2, 20) for st in (True, False)}
    r.update({f"tick{k}_devsync": tm(tk(k, True, True)) for k in (1, 20)})
    print("split", split, r)
    if split == "1" and os.environ.get("PROBE_COMM") == "1":   # single-rank RCCL communicator (the N>1 stats path)
        e.comm_init(1, 0, Engine.comm_unique_id())
        print("split 1 comm", {f"tick{k}_devsync": tm(tk(k, True, True)) for k in (1, 20)})
    e.close()
