"""Kernel span and wall time of steady calls with and without statistics
(profile mode 1: one event pair spanning each call's launches), alternating,
on one engine: does per-tick statistics collection slow the tick kernel?

    python tools/stats_cost.py [--workload C2X] [--calls 4] [--steps 20]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raft-sample_amd"))
import bench  # noqa: E402
from raftstep import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C2X")
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    R, G, K, E, crc = wl.get("replicas", 5), wl["groups"], wl["ring_depth"], wl["entries"], wl["crc"]
    e = Engine(**bench.engine_kwargs(wl, R, G, 0, K, E, crc))
    e.init_steady(0, 0)
    t = 1
    e.tick(t, 5)
    t += 5
    e.tick(t, a.steps)
    t += a.steps
    for c in range(a.calls):
        for st in (False, True):
            e.profile(1)
            t0 = time.perf_counter()
            e.tick(t, a.steps, stats=st)
            e.sync()
            wall = (time.perf_counter() - t0) * 1e6 / a.steps
            ms, n = e.profile_read()
            e.profile(0)
            t += a.steps
            print(f"call {c} stats={int(st)}: kernel span {ms * 1e3 / a.steps:7.1f} us/tick, wall {wall:7.1f} us/tick",
                  flush=True)


if __name__ == "__main__":
    main()
