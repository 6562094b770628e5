"""Summarise rocprofv3 --pmc passes into per-launch HBM traffic.

Usage (after the GPU session wrote the pass directories):
    python tools/pmc_summary.py --calib-fetch DIR --calib-write DIR \
        --fetch DIR --write DIR --kernel tick_fast_kernel --workload "..." --out profiles/pmc_latest.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. Per MI355X_MICROARCH.md
§HBM they are only calibrated for 16-B/lane streams, so each is divided by
the ratio counter/true-bytes measured by tools/pmc_calib (same access widths
as the tick kernels: 4-B and 8-B per lane, coalesced, 1 GiB per kernel).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

CALIB_BYTES = 1 << 30


def load(dirpath, counter):
    """{kernel_name: [values per dispatch]} for one counter."""
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {dirpath}")
    per = defaultdict(lambda: defaultdict(float))
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            disp = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            per[name][disp] += float(row["Counter_Value"])
    return {k: [v[i] for i in sorted(v)] for k, v in per.items()}


def mean_for(d, key, skip=0, take=None):
    """Mean over the dispatches of the kernels whose name contains `key`, in
    dispatch order, after the first `skip` (e.g. settle and warm-up ticks),
    at most `take` of them."""
    vals = [v for k, vs in d.items() if key in k for v in vs]
    vals = vals[skip:skip + take] if take else vals[skip:]
    if not vals:
        raise SystemExit(f"kernel {key!r} not found in {list(d)}")
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="tick_fast_kernel")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--algorithmic-bytes", type=float, default=None)
    ap.add_argument("--commit", default=None, help="git commit of the build the passes ran on")
    ap.add_argument("--ticks-per-launch", type=float, default=1,
                    help="ticks one launch of the kernel ran (tick_fused_kernel); bench.py matches on it")
    ap.add_argument("--launches-per-tick", type=int, default=1,
                    help="dispatches of the kernel per tick (2: the split steady tick's two halves)")
    ap.add_argument("--skip", type=int, default=0, help="leave out the kernel's first SKIP dispatches (settle, warm-up)")
    ap.add_argument("--take", type=int, default=None, help="then average at most TAKE dispatches (the timed call)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    cf, cw = load(a.calib_fetch, "FETCH_SIZE"), load(a.calib_write, "WRITE_SIZE")
    calib = {}
    for k in ("read_u32", "read_u64"):
        calib[k] = mean_for(cf, k)[0] * 1024 / CALIB_BYTES
    for k in ("write_u32", "write_u64"):
        calib[k] = mean_for(cw, k)[0] * 1024 / CALIB_BYTES
    read_corr = calib["read_u32"]
    write_corr = (calib["write_u32"] + calib["write_u64"]) / 2
    f_kb, nf = mean_for(load(a.fetch, "FETCH_SIZE"), a.kernel, a.skip, a.take)
    w_kb, nw = mean_for(load(a.write, "WRITE_SIZE"), a.kernel, a.skip, a.take)
    rd = f_kb * 1024 / read_corr
    wr = w_kb * 1024 / write_corr
    out = {
        "workload": a.workload, "kernel": a.kernel, "dispatches": [nf, nw],
        "fetch_kib_per_launch": f_kb, "write_kib_per_launch": w_kb,
        "calibration_counter_over_true": calib, "read_corr": read_corr, "write_corr": write_corr,
        "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
    }
    out["launches_per_tick"] = a.launches_per_tick
    out["hbm_bytes_per_tick"] = (rd + wr) * a.launches_per_tick
    if a.algorithmic_bytes:   # (per launch)
        out["traffic_over_algorithmic"] = (rd + wr) / a.algorithmic_bytes
    out["ticks_per_launch"] = a.ticks_per_launch
    out["dispatch_window"] = {"skip": a.skip, "take": a.take}
    if a.commit:
        out["commit"] = a.commit
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
