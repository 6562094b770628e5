"""Per-tick lane-class counts (raft_diag_read) of a workload in bench.py's
timed region: settle + warm-up as the bench, then TICKS ticks with the class
counters on (their atomics slow the kernels; counts only).
    python tools/classes.py [--workload C4] [--ticks 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raft-sample_amd")]
import bench  # noqa: E402
from raftstep import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="C4")
ap.add_argument("--ticks", type=int, default=20)
a = ap.parse_args()
wl = bench.WORKLOADS[a.workload]
R = wl.get("replicas", 5)
e = Engine(**bench.engine_kwargs(wl, R, wl["groups"], 0, wl["ring_depth"], wl["entries"], wl["crc"]))
if wl.get("init") == "new":
    e.init_new_nodes(0)
    e.tick(0, wl["settle"])
    t = wl["settle"]
else:
    e.init_steady(0, 0)
    t = 1
e.tick(t, 5)
t += 5
e.diag_enable(True)
e.tick(t, a.ticks)
import ctypes as C  # noqa: E402
from raftstep import abi  # noqa: E402
buf = (C.c_uint64 * abi.DIAG_COUNTERS)()
e.lib.raft_diag_read(e.h, buf, abi.DIAG_COUNTERS)
names = {i: k for k, i in abi.DIAG.items()}
# (a DIAG=1 build also counts deferral reasons: list slots 43-47)
reasons = {43: "defer_reason_not_steady", 44: "defer_reason_iso", 45: "defer_reason_follower_out_of_step",
           46: "defer_reason_rows_out_of_step", 47: "defer_reason_later"}
c = {names.get(i, reasons.get(i, f"slot{i}")): int(buf[i]) for i in range(abi.DIAG_COUNTERS)}
c["general_worklist_note"] = "general_launches counts windows"
print(json.dumps({k: (v / a.ticks if isinstance(v, int) else v) for k, v in sorted(c.items(), key=lambda kv: str(kv[1])) if v},
                 indent=1))
