"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, restricted to a
window of each kernel's dispatches (e.g. the bench's timed call), next to the
whole-run mean rocprofv3 --stats reports.

    python tools/trace_summary.py TRACE.csv --skip-ticks S --ticks N [--launches-per-tick L] [--out F]

A tick is L tick_lean_kernel dispatches (2 for the split steady tick, whose
halves run on two streams); the window is the N ticks after the first S
dispatches (settle + warm-up), and every other kernel is counted inside the
time span of those ticks' lean dispatches."""
import argparse
import csv
import json
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("raftstep::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-ticks", type=int, required=True)
    ap.add_argument("--ticks", type=int, required=True)
    ap.add_argument("--launches-per-tick", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
    lean = [x for x in k if x[2].startswith("tick_lean_kernel") or x[2].startswith("tick_fused_kernel")]
    win = lean[a.skip_ticks:a.skip_ticks + a.ticks * a.launches_per_tick]
    t0, t1 = min(x[0] for x in win), max(x[1] for x in win)
    per = defaultdict(list)
    for s, e, n in k:
        if s >= t0 and e <= t1 + 1:
            per[n].append(e - s)
    allk = defaultdict(list)
    for s, e, n in k:
        allk[n].append(e - s)
    out = {"trace": a.trace, "window": {"skip_ticks": a.skip_ticks, "ticks": a.ticks,
                                        "span_us": (t1 - t0) / 1e3, "us_per_tick": (t1 - t0) / 1e3 / a.ticks},
           "kernels": {n: {"window_dispatches": len(v), "window_mean_us": sum(v) / len(v) / 1e3,
                           "run_dispatches": len(allk[n]), "run_mean_us": sum(allk[n]) / len(allk[n]) / 1e3}
                       for n, v in sorted(per.items())}}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
