"""Interleaved in-process A/B of engine variants (methodology rule 24 of
cdna_hip_programming.md: one process, interleaved rounds, report median/min).

Variants are env knobs read at engine creation:
  RAFTSTEP_WRITE_THROUGH=1   fast-kernel stores with sc1 (write-through)
  RAFTSTEP_SLOW_EVERY=N      general kernel every N ticks

    python tools/ab.py --groups 1048576 --ticks 100 --rounds 5 \
        base: wt:RAFTSTEP_WRITE_THROUGH=1 se32:RAFTSTEP_SLOW_EVERY=32
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-sample_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1 << 20)
    ap.add_argument("--replicas", type=int, default=5)
    ap.add_argument("--ticks", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--noprof", action="store_true", help="no per-kernel events (wall time only)")
    ap.add_argument("variants", nargs="+", help="name:K=V,K=V")
    a = ap.parse_args()
    from raftstep import Engine
    engines = {}
    for spec in a.variants:
        name, _, kv = spec.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            e = Engine(replicas=a.replicas, groups=a.groups, ring_depth=32, client_period=1, seed=0x5EED0002)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        e.init_steady(0, 0)
        e.tick(1, 10)
        engines[name] = [e, 11]
    res = {n: {"wall_us": [], "kern_us": []} for n in engines}
    for _ in range(a.rounds):
        for n, (e, t) in engines.items():
            e.sync()
            e.profile(2 if a.noprof else 1)
            t0 = time.perf_counter()
            e.tick(t, a.ticks, stats=False)
            e.sync()
            dt = time.perf_counter() - t0
            ms, k = e.profile_read()
            e.profile(0)
            engines[n][1] = t + a.ticks
            res[n]["wall_us"].append(dt * 1e6 / a.ticks)
            res[n]["kern_us"].append(ms * 1e3 / max(k, 1))
    out = {n: {k: {"median": statistics.median(v), "min": min(v)} for k, v in d.items()} for n, d in res.items()}
    print(json.dumps({"groups": a.groups, "ticks": a.ticks, "rounds": a.rounds, "results": out}))


if __name__ == "__main__":
    main()
