"""Per-kernel averages of a rocprofv3 --pmc counter CSV (per-wave figures)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(d, "no counter csv")
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        agg[r["Kernel_Name"].split("(")[0][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "tick" not in k and "probe" not in k:
            continue
        avg = {c: sum(x) / len(x) for c, x in v.items()}
        w = max(avg.get("SQ_WAVES", 1), 1)
        print(k, "launches", len(next(iter(v.values()))), " ".join(f"{c[3:]}={avg[c]/w:.1f}" for c in sorted(avg) if c != "SQ_WAVES"),
              f"waves={w:.0f}")
