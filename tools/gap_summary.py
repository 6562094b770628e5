"""Gaps between a kernel's end and the next dispatch's start in a rocprofv3
kernel trace (diagnostics for tools/gap_probe.hip): median per (kernel, grid).

    python tools/gap_summary.py <run_kernel_trace.csv>
"""
import csv
import statistics
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    for a, b in zip(rows, rows[1:]):
        if not a["Kernel_Name"].startswith("void dirty"):
            continue
        key = (a["Kernel_Name"].split("(")[0], int(a["Grid_Size_X"]))
        dur = (int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1000
        gap = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000
        out.setdefault(key, []).append((dur, gap))
    for (k, grid), v in sorted(out.items()):
        v = v[2:]   # first rounds: warm-up
        print(f"{k:28s} grid {grid:>10d}  kernel {statistics.median(x[0] for x in v):8.1f} us"
              f"  gap to next {statistics.median(x[1] for x in v):7.1f} us  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
