"""Summarise bench JSON lines: value, ms/step, lean / list kernel us, region us."""
import glob
import json
import sys

for pat in sys.argv[1:]:
    for f in sorted(glob.glob(pat)):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except Exception as e:   # noqa: BLE001
            print(f, "unreadable:", e)
            continue
        r = d["roofline"]
        print(f"{f.split('/')[-1]:28s} {d['value']:.3e} ms/step {d['ms_per_step']:.4f} lean {r['avg_kernel_us']:.1f} "
              f"list {r['list_kernel_us'] or 0:.1f} region {r['avg_region_us_per_tick']:.1f} frac {r['frac']:.3f} ok {d['stats_check']}")
