"""Print one line per bench JSON log: value, per-repeat ms/step, kernel us."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except (IndexError, OSError, ValueError) as e:
        print(f, "no result", e)
        continue
    r = d["roofline"]
    print(f"{f}: {d['value']:.3e} ms/step {[round(x, 4) for x in d['timing']['repeat_ms_per_step']]} "
          f"kern {r['avg_kernel_us']:.1f} us frac {r['frac']:.3f} ok {d['stats_check']}")
