"""Timing-only diagnostics of the C4 lean and list kernels (results are WRONG
in the diag modes; never a bench line): for each diagnostic mode (0 = the
product kernels; lean: 4 = whole ring rows written, no holes, 8 = no
stale-column writes; list: 32 = staging alone, 64 = staging and write-back,
128 = the per-group code alone, 256 = no list work, 512 = no entry copies or
moves) and pipeline on/off, the lean and list kernels' mean durations and the
tick's wall time over TICKS ticks. The mode is switched on after the bench's
settle and warm-up ticks (raft_debug_diag_mode), so those run exactly and the
measured ticks start from the benchmark's state.
    python tools/lean_diag.py [--workload C4] [--modes 0,4] [--pipeline 1,0]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raft-sample_amd")]
import bench  # noqa: E402
from raftstep import Engine, abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="C4")
ap.add_argument("--modes", default="0,4")
ap.add_argument("--pipeline", default="1,0")
ap.add_argument("--ticks", type=int, default=20)
a = ap.parse_args()
wl = bench.WORKLOADS[a.workload]
R = wl.get("replicas", 5)
out = []
for pipe in a.pipeline.split(","):
    for mode in a.modes.split(","):
        os.environ["RAFTSTEP_PIPELINE"] = pipe
        e = Engine(debug_flags=abi.DEBUG_ALLOW_WRONG_RESULTS,
                   **bench.engine_kwargs(wl, R, wl["groups"], 0, wl["ring_depth"], wl["entries"], wl["crc"]))
        e.init_new_nodes(0)
        e.tick(0, wl["settle"])
        t = wl["settle"]
        e.tick(t, 5)
        t += 5
        e.debug_diag_mode(int(mode))
        e.sync()
        t0 = time.perf_counter()
        e.tick(t, a.ticks)
        wall = (time.perf_counter() - t0) / a.ticks
        t += a.ticks
        e.profile(1)
        e.tick(t, a.ticks, stats=False)
        t += a.ticks
        lms, ln = e.profile_read()
        e.profile(3)
        e.tick(t, a.ticks, stats=False)
        lsm, lsn = e.profile_read()
        e.profile(0)
        e.close()
        out.append({"pipeline": pipe, "diag": mode, "tick_us": wall * 1e6, "lean_us": lms * 1e3 / max(ln, 1),
                    "list_us": lsm * 1e3 / max(lsn, 1)})
        print(json.dumps(out[-1]), flush=True)

