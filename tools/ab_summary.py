"""Summarise an A/B directory written by tools/gpu_ab.sh: value and kernel
times per variant (each round), medians."""
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
rows = defaultdict(list)
for p in sorted(glob.glob(os.path.join(d, "*_*.json"))):
    v = os.path.basename(p).rsplit("_", 1)[0]
    try:
        x = json.load(open(p))
    except ValueError:
        continue
    ro = x["roofline"]
    lk = x.get("list_kernel") or {}
    rows[v].append((x["value"], ro["avg_kernel_us"], lk.get("avg_us"), x["ms_per_step"]))
for v, rs in rows.items():
    med = sorted(r[0] for r in rs)[len(rs) // 2]
    print(f"{v:12s} median {med:.4g}  " + "  ".join(
        f"[{r[0]:.4g} lean {r[1]:.1f} list {r[2] if r[2] is None else round(r[2], 1)} ms/t {r[3]:.4f}]" for r in rs))
