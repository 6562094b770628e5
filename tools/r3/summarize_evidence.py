"""After tools/r3/gpu_evidence.sh: per-launch HBM traffic of the tick kernels
from the FETCH_SIZE / WRITE_SIZE passes (tools/pmc_summary.py), written to
profiles/pmc_<workload>[_<kernel>].json with the workload string of the same
session's bench line (what bench.py's load_pmc matches), and a copy of the
session's bench lines, kernel-trace summaries and logs under profiles/r03/<name>/.

    python tools/r3/summarize_evidence.py gpurun_out/r3ev final <commit>
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src, name, commit = sys.argv[1], sys.argv[2], sys.argv[3]
dst = os.path.join(ROOT, "profiles", "r03", name)
os.makedirs(dst, exist_ok=True)


def tpl(line):
    """Mean ticks per launch of the line's calls (bench.py: --steps over ceil(steps / depth) launches)."""
    r = line["roofline"]
    t = r.get("max_ticks_per_launch", r.get("ticks_per_launch", 1))
    return line["steps"] / -(-line["steps"] // t) if t > 1 else 1


def bench_line(f):
    return json.loads(open(os.path.join(src, f)).read().strip().splitlines()[-1])


passes = {   # workload tag -> (bench line, pmc pass prefix, kernels); the first is the line's roofline kernel
    "C2": ("bench_c2.json", "pmc_c2", ["tick_fused_kernel"]),
    "C2_4M": ("bench_c2_4m.json", "pmc_c2_4m", ["tick_fused_kernel"]),
    "C3": ("bench_c3.json", "pmc_c3", ["tick_fused_kernel"]),
    "C4": ("bench_c4.json", "pmc_c4", ["tick_lean_kernel", "tick_list_kernel", "tick_seg_kernel"]),
    "C5": ("bench_c5.json", "pmc_c5", ["tick_lean_kernel"]),
}
for tag, (bf, pre, kernels) in passes.items():
    if not os.path.exists(os.path.join(src, pre + "_write")):
        print(f"{tag}: no PMC passes in {src}, kept as is")
        continue
    line = bench_line(bf)
    for k in kernels:
        main = k == kernels[0]
        out = os.path.join(ROOT, "profiles", f"pmc_{tag}.json" if main else f"pmc_{tag}_{k[5:]}.json")
        cmd = [sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"),
               "--calib-fetch", os.path.join(src, "pmc_calib_fetch"), "--calib-write", os.path.join(src, "pmc_calib_write"),
               "--fetch", os.path.join(src, pre + "_fetch"), "--write", os.path.join(src, pre + "_write"),
               "--kernel", k, "--workload", line["config"]["workload"], "--commit", commit, "--out", out,
               "--ticks-per-launch", str(tpl(line) if main else 1)]
        if main:   # (bytes per tick x mean ticks per launch: the passes count per launch)
            r = line["roofline"]
            t = r.get("ticks_per_launch", 1)
            B = r["bytes_per_group_step"]
            if "max_ticks_per_launch" not in r and t > 1:   # (older lines: priced at the full depth, 40 B per launch)
                n = -(-line["steps"] // t)
                B, t = B - 40 / t + 40 * n / line["steps"], line["steps"] / n
            cmd += ["--algorithmic-bytes", str(B * r["units_per_launch"] * t)]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
        d = json.load(open(out))
        print(f"{tag:6s} {k:18s} {d['hbm_bytes_per_launch'] / 1e6:9.1f} MB/launch", d.get("traffic_over_algorithmic", ""))
for f in sorted(os.listdir(src)):
    p = os.path.join(src, f)
    if f.endswith((".json", ".log")) and os.path.isfile(p):
        shutil.copy(p, dst)
for prof in ("prof_c2", "prof_c4"):
    for root, _, files in os.walk(os.path.join(src, prof)):
        for f in files:
            if f.endswith("kernel_stats.csv"):
                shutil.copy(os.path.join(root, f), os.path.join(dst, f"{prof[5:]}_kernel_stats.csv"))
print("copied to", dst)
