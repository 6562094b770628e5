"""Prints the headline and per-workload numbers of a bench.py JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(d["config"]["workload"][:40], "value %.4g" % d["value"], "frac %.3f" % r["frac"], "lean_us %.1f" % r["avg_kernel_us_per_tick"],
      "check", d["stats_check"], "list_us", (d.get("list_kernel") or {}).get("avg_us"))
for k, x in (d.get("extra_workloads") or {}).items():
    if "value" not in x:
        print(k, x)
        continue
    print(k, "value %.4g" % x["value"], "frac %.3f" % x["roofline"]["frac"], "lean_us %.1f" % x["roofline"]["avg_kernel_us_per_tick"],
          "check", x["stats_check"], "list_us", (x.get("list_kernel") or {}).get("avg_us"),
          "pcie", (x.get("pcie_inclusive") or {}).get("value"), "rej", (x.get("verification") or {}).get("rejections"),
          "stats", x["stats"])
print("wall", d.get("bench_wall_s"))
