"""Where a C4 list-kernel wave spends its time (diagnostics build only):
    tools/ablib.sh wprof -DRAFTSTEP_WAVE_PROF
    RAFTSTEP_LIB=ablib/wprof/libraftstep.so python tools/list_prof.py [--workload C4]
Runs the workload as bench.py does (settle, warm-up), then TICKS ticks with
the device counters on; the list kernel's lane 0 of every wave adds its
phase cycles (s_memtime) there (k_fast.hip RAFTSTEP_WAVE_PROF)."""
import argparse
import ctypes as C
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
G = wl["groups"]
e = Engine(**bench.engine_kwargs(wl, R, G, 0, wl["ring_depth"], wl["entries"], wl["crc"]))


def run(t, k, **kw):   # (staged workloads: this call's values first)
    if wl.get("staged"):
        e.stage_values(t, bench.staged_values(wl["seed"], 0, G, t, k, wl["entries"]))
    e.tick(t, k, **kw)
    return t + k


if wl.get("init") == "new":
    e.init_new_nodes(0)
    t = run(0, wl["settle"])
else:
    e.init_steady(0, 0)
    t = 1
t = run(t, 5)
e.profile(3)
t = run(t, a.ticks, stats=False)
lms, ln = e.profile_read()
e.profile(0)
e.diag_enable(True)
t = run(t, a.ticks, stats=False)
buf = (C.c_uint64 * 72)()
e.lib.raft_diag_read(e.h, buf, 72)
d = list(buf)
waves = max(d[4], 1)
steps = max(d[37], 1)
out = {"list_kernel_us_mean": lms * 1e3 / max(ln, 1), "launches": ln, "waves_per_launch": d[4] / a.ticks,
       "max_wave_cycles": d[5],
       "per_wave_cycles": {"staging": d[0] / waves, "step1": d[1] / waves, "step2": d[2] / waves,
                           "write_back": d[3] / waves},
       "per_step_cycles": {"per_group_code": d[32] / steps, "copy_gather": d[33] / steps,
                           "own_ring_writes": d[34] / steps, "copy_scatter": d[35] / steps,
                           "worklist_stats": d[36] / steps},
       "wave_cycles_log2_hist": {f"2^{k + 10}": d[6 + k] for k in range(16) if d[6 + k]}}
print(json.dumps(out, indent=1))
