"""Benchmark: Raft group-steps/sec (BASELINE.json metric) on MI355X.

One step = one tick of every group: client append of E
entries to the leader (main.go:327-329), one leader replication round to all
R-1 peers through their AppendEntries handlers (main.go:334-379, 121-156),
the commit rule (main.go:381-391) and the election timers — one fused kernel
launch per tick, state read from and written back to HBM every tick.

Workload at N=1: SURVEY config C2 — 2^20 independent 5-replica groups,
steady-state AppendEntries + commitIndex, one client entry per tick, seeded
synthetic trace. For N>1 the default is SURVEY config C3: each rank owns
2^21 groups (16M over 8 GPUs; weak scaling; groups shard by id, no
data-path collective); the per-tick statistics are reduced on the device and
summed across GPUs with RCCL on a side stream inside the engine.

Protocol: W untimed warm-up ticks, then the timed region of
exactly K ticks (barrier + synchronize on both sides, max over ranks) is
repeated --repeats times (default 5) and the median is reported. The
roofline's `achieved` uses the steady-state kernel's own average duration,
measured by HIP events attached to each of its dispatches (profile mode 1)
in a separate, untimed pass of K ticks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C2|C3|C4|C4R|C4REF|C5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-sample_amd"))

R_DEFAULT = 5
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(R, E, crc=False):
    """minimal SoA bytes per group-step, REF steady state:
    B(R,E) = 25 + 37(R-1) + 12 E R (233 B at R=5, E=1), + 4 E R with a
    CRC32C stamp per entry (C5: 5293 B). This is the per-replica SoA
    accounting (every replica's term/last/commit/deadline and every peer's
    MatchIndex read and written each tick); the compressed steady state
    needs less (lean_bytes), so the SURVEY figure is reported as an
    equivalent rate, never against the HBM peak."""
    return 25 + 37 * (R - 1) + 12 * E * R + (4 * E * R if crc else 0)


def fused_ticks(wl):
    """Ticks per launch of the steady-state tick (engine.cpp raft_engine::fuse):
    RAFTSTEP_FUSE (default 16) while the steady-state list skip holds — the
    steady workloads without payload CRC — else 1."""
    if wl.get("init") == "new" or wl["crc"] or os.environ.get("RAFTSTEP_TWO_PASS", "1") == "0":
        return 1
    return max(1, int(os.environ.get("RAFTSTEP_FUSE", "16")))


def lean_bytes(R, E, crc=False, segmented=False, fuse=1):
    """Algorithmic bytes per group-step of tick_lean_kernel (the dominant
    kernel of the two-pass tick, k_fast.hip) in this engine's layout: a group
    in the compressed steady state (SSYNC) holds term / LastApplied / the
    leader's and the followers' CommitIndex in one 16-B record, MatchIndex
    rows and follower timers are implicit (MSYNC, hb). Per group-step it
    reads gmeta 2 B + the record 16 B + the ring rotation 2 B (+ the ring
    segment boundary 4 B when the ring has 2K physical slots) and writes the
    record 16 B + hb 4 B + this tick's entries on all R replicas, 12 E R B
    (+4 E R with a CRC32C stamp). C2: 100 B; C4 shape (R=7, 2K slots): 128 B;
    C5: 5160 B. With `fuse` ticks per launch (tick_fused_kernel) the
    record / meta / rotation / heartbeat bytes are moved once per launch:
    40 / fuse + 12 E R (C2 at 4 ticks per launch: 70 B)."""
    return (20 + (4 if segmented else 0) + 20) / fuse + 12 * E * R + (4 * E * R if crc else 0)


# SURVEY.md §8(d) workloads runnable by this bench (per GPU)
WORKLOADS = {
    "C2": dict(groups=1 << 20, entries=1, ring_depth=32, crc=0, seed=0x5EED0002,
               desc="steady-state AppendEntries+commit"),
    "C3": dict(groups=1 << 21, entries=1, ring_depth=32, crc=0, seed=0x5EED0003,
               desc="steady-state AppendEntries+commit, 2^21 groups per GPU (16M over 8 GPUs)"),
    "C5": dict(groups=1 << 20, entries=64, ring_depth=128, crc=1, seed=0x5EED0005,
               desc="64-entry AppendEntries batches with per-entry CRC32C stamp+verify"),
    # C4: NewNode start, leader isolation: per 32-tick epoch
    # w.p. 1/8 (~1/256 per tick) a window of 8-32 ticks cuts off the group's
    # leader (the lowest-id Leader at the window's first tick); RAFT semantics
    # (REF faults on a new leader's first contact, SURVEY KAT-11)
    "C4": dict(groups=1 << 22, replicas=7, entries=1, ring_depth=128, crc=0, init="new", semantics=1, settle=48,
               iso=(8192, 8, 32, 1), seed=0x5EED0004,
               desc="NewNode start, leader-isolation churn (elections, step-downs, truncation), RAFT semantics"),
    # C4R: the same with the isolated replica drawn from the trace hash (any
    # replica; the leader 1 time in 7) -- round 1's C4 line
    "C4R": dict(groups=1 << 22, replicas=7, entries=1, ring_depth=128, crc=0, init="new", semantics=1, settle=48,
                iso=(8192, 8, 32, 0), seed=0x5EED0004,
                desc="NewNode start, hashed-replica isolation churn, RAFT semantics"),
    # C4REF: C4's trace in REF semantics (main.go bit for bit): the first
    # contact of a new leader panics (GetLog, main.go:142 -> 404) and the
    # group freezes, so this line reports throughput over the prefix and the
    # fault counts (SURVEY §8(d) "REF parity on prefix + fault codes")
    "C4REF": dict(groups=1 << 22, replicas=7, entries=1, ring_depth=128, crc=0, init="new", semantics=0, settle=48,
                  iso=(8192, 8, 32, 1), seed=0x5EED0004, allow_faults=True,
                  desc="NewNode start, leader-isolation churn, REF semantics (prefix; groups freeze on their first fault)"),
}


def cpu_baseline(args, wl, R, E, K, crc):
    """The oracle (C restatement of main.go's handlers, oracle/) timed on the
    host cores on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    G, T = args.cpu_groups, args.cpu_ticks
    if E > 1:   # keep the sample's CPU time and memory bounded for big batches
        G, T = max(1024, 4 * G // E), max(16, T // 4)
    o = oracle.Oracle(**engine_kwargs(wl, R, G, 0, K, E, crc))
    if wl.get("init") == "new":
        G, T = G // 2, T // 2
        o.close()
        o = oracle.Oracle(**engine_kwargs(wl, R, G, 0, K, E, crc))
        o.init_new_nodes(0)
        o.tick(0, wl["settle"], threads=threads)
        t_first, start = wl["settle"], "after a NewNode start and %d settle ticks" % wl["settle"]
    else:
        o.init_steady(0, 0)
        t_first, start = 1, "steady state from init_steady"
    t0 = time.perf_counter()
    o.tick(t_first, T, threads=threads)
    dt = time.perf_counter() - t0
    o.close()
    return {"value": G * T / dt, "unit": "group-steps/s", "cores": threads, "kind": "port",
            "sample": f"G scaled down to {G} groups (GPU line: {wl['groups']}) x {T} ticks, R={R}, E={E}, "
                      f"crc={crc}, {start}; oracle/raft_oracle.c (C restatement of main.go's handlers), "
                      f"{threads} pthreads over contiguous group ranges ({dt:.2f} s)"}


def engine_kwargs(wl, R, G, base, K, E, crc):
    kw = dict(replicas=R, groups=G, group_base=base, ring_depth=K, entries_per_tick=E, client_period=1,
              payload_crc=crc, seed=wl["seed"], semantics=wl.get("semantics", 0))
    if "iso" in wl:
        kw.update(isolate_per_65536=wl["iso"][0], isolate_min_ticks=wl["iso"][1], isolate_max_ticks=wl["iso"][2],
                  isolate_leader=wl["iso"][3])
    return kw


def load_pmc(workload, kernel, ticks=1):
    """HBM traffic per launch of the dominant kernel from the committed
    rocprofv3 --pmc summary of exactly this workload, kernel and ticks per
    launch (mean over the pass's launches; profiles/pmc_*.json, made by tools/pmc_summary.py from FETCH_SIZE /
    WRITE_SIZE passes), and where it came from; (None, None) if no pass
    covers it."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("kernel") == kernel and d.get("hbm_bytes_per_launch") and \
                abs(d.get("ticks_per_launch", 1) - ticks) < 1e-6:
            src = f"{os.path.relpath(p, ROOT)} (rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes of this workload, " \
                  f"calibrated by tools/pmc_calib; not measured in this run" + \
                  (f"; build {d['commit']}" if d.get("commit") else "") + ")"
            return d["hbm_bytes_per_launch"], src
    return None, None


def median(xs):
    xs = sorted(xs)
    n = len(xs)
    return xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--repeats", type=int, default=5, help="timed regions of --steps ticks; the median is reported")
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: C2 at --gpus 1, C3 (2^21 groups per GPU) at --gpus > 1")
    ap.add_argument("--groups-per-gpu", type=int, default=None)
    ap.add_argument("--replicas", type=int, default=None)
    ap.add_argument("--entries", type=int, default=None)
    ap.add_argument("--ring-depth", type=int, default=None)
    ap.add_argument("--leader", type=int, default=0, help="steady-state leader replica (-1: hashed per group)")
    ap.add_argument("--cpu-groups", type=int, default=262144)
    ap.add_argument("--cpu-ticks", type=int, default=1024)   # ~10 s of oracle work on 16 host threads
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--isolate", type=int, default=None,
                    help="diagnostics: override the workload's isolation windows per 65536 epochs (0: none)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    wl_key = args.workload or ("C2" if world == 1 else "C3")

    import torch
    dist = None
    # test hook: several ranks on ONE GPU (gloo for torch.distributed, no engine
    # RCCL communicator) to rehearse the N>1 path on a one-GPU box
    same_dev = os.environ.get("RAFTSTEP_BENCH_SAME_DEVICE") == "1"
    if same_dev:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if same_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from raftstep import Engine, STAT_NAMES

    wl = WORKLOADS[wl_key]
    if args.isolate is not None and "iso" in wl:
        wl = dict(wl, iso=(args.isolate,) + tuple(wl["iso"][1:]))
    R = args.replicas or wl.get("replicas", R_DEFAULT)
    G = args.groups_per_gpu or wl["groups"]
    E = args.entries or wl["entries"]
    K = args.ring_depth or wl["ring_depth"]
    crc = wl["crc"]
    churn = wl.get("init") == "new"
    base = rank * G
    eng = Engine(device=local, **engine_kwargs(wl, R, G, base, K, E, crc))
    if dist is not None and not same_dev:
        from raftstep import dist as rdist
        eng.comm_init(world, rank, rdist.exchange_comm_id(dist, rank, Engine.comm_unique_id))
    untimed = np.zeros(len(STAT_NAMES), np.int64)   # stats of the settle and warm-up ticks
    if churn:   # NewNode start; the first elections happen in untimed settle ticks
        eng.init_new_nodes(0)
        untimed += eng.tick(0, wl["settle"], stats=True)
        tick = wl["settle"]
    else:
        eng.init_steady(args.leader, 0)
        tick = 1
    if args.warmup:
        untimed += eng.tick(tick, args.warmup, stats=True)
        tick += args.warmup

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # timed regions: exactly K fused ticks each (+ the per-tick stats, reduced
    # on the device and, at N>1, all-reduced by RCCL on the engine's side stream)
    times, stats = [], np.zeros(len(STAT_NAMES), np.int64)
    # groups frozen by a fault before each tick (REF prefix: a frozen group does
    # no work, so C4REF's value counts only the live group-steps)
    frozen = int(untimed[STAT_NAMES.index("faults")])
    live_steps = []
    eng.profile(2)   # one HIP event pair on the engine stream around each timed call
    for _ in range(max(1, args.repeats)):
        barrier()
        t0 = time.perf_counter()
        s = eng.tick(tick, args.steps, stats=True)
        barrier()
        el = time.perf_counter() - t0
        if wl.get("allow_faults"):   # (outside the timed region) per-tick fault counts of this rank
            f = eng.tick_records(args.steps)[:, STAT_NAMES.index("faults")]
            before = frozen + np.concatenate([[0], np.cumsum(f)[:-1]])
            live_steps.append(int(G * args.steps - before.sum()))
            frozen += int(f.sum())
        if dist is not None:
            from raftstep import dist as rdist
            el = rdist.max_over_ranks(dist, el, device=None if same_dev else "cuda")
            if same_dev:   # no engine communicator: sum the stats through torch.distributed
                s = np.array(rdist.sum_over_ranks(dist, s), np.int64)
        times.append(el)
        stats += s
        tick += args.steps
    region_ms, region_launches = eng.profile_read()
    # untimed pass: the steady-state kernel's own duration, events attached to each dispatch
    eng.profile(1)
    eng.tick(tick, args.steps, stats=False)
    kernel_ms, kernel_launches = eng.profile_read()
    two_pass = os.environ.get("RAFTSTEP_TWO_PASS", "1") != "0"
    list_ms = list_launches = 0
    if two_pass:   # the second pass (list kernel over the groups the lean kernel passed on)
        eng.profile(3)
        eng.tick(tick + args.steps, args.steps, stats=False)
        list_ms, list_launches = eng.profile_read()
    eng.profile(0)
    nranks, _, allreduces = eng.comm_info()

    elapsed = median(times)
    reps = len(times)
    total_steps = G * world * args.steps
    value = total_steps / elapsed
    live_value = None
    if wl.get("allow_faults"):   # C4REF: only the group-steps of groups not frozen by a fault count
        mid = sorted(range(reps), key=lambda i: times[i])[reps // 2]
        live = live_steps[mid]
        if dist is not None:
            from raftstep import dist as rdist
            live = int(sum(rdist.sum_over_ranks(dist, [live])))
        live_value = live / times[mid]
        value = live_value
    # correctness guard on the timed runs: the steady state commits exactly one
    # entry per group per tick and never faults; under churn nothing faults
    # and most groups have a leader (REF prefix: faults are the point)
    expect_commit = G * world * args.steps * E * reps
    faults = int(stats[STAT_NAMES.index("faults")])
    if churn:
        ok = (wl.get("allow_faults") or faults == 0) and \
            (wl.get("allow_faults") or stats[STAT_NAMES.index("leader_groups")] > 0.5 * G * world * args.steps * reps)
    else:
        ok = stats[STAT_NAMES.index("committed")] == expect_commit and faults == 0
    if world > 1 and not same_dev:
        # the engine communicator must span every rank, and every window's
        # stats must have gone through it (ncclAllReduce on the side stream)
        if nranks != world:
            raise SystemExit(f"bench: RCCL communicator has {nranks} ranks, WORLD_SIZE is {world}")
        ok = ok and allreduces > 0

    B_survey = algorithmic_bytes(R, E, crc)
    # the dominant kernel's algorithmic bytes in its own layout: the lean
    # kernel (compressed steady state) in the two-pass tick, else the
    # one-pass fast kernel with SURVEY §8(d)'s per-replica SoA accounting
    fuse = fused_ticks(wl)
    # a call of K ticks runs ceil(K / fuse) fused launches (K = 20: 16 + 4);
    # the bytes moved once per launch are priced at the mean ticks per launch
    tpl = args.steps / -(-args.steps // fuse) if fuse > 1 else 1
    B = lean_bytes(R, E, crc, segmented="iso" in wl and wl["iso"][0] > 0, fuse=tpl) if two_pass else B_survey
    avg_kernel_s = kernel_ms / 1e3 / max(kernel_launches, 1)    # steady-state kernel, kernel-exact
    avg_region_s = region_ms / 1e3 / max(region_launches, 1)    # all launches of a tick + gaps
    # C4REF: the lean kernel's algorithmic bytes are those of the live groups it
    # takes (a frozen group is read as 2 B of gmeta and skipped)
    units = G if live_value is None else live_value * elapsed / world / args.steps
    achieved = B * units / avg_kernel_s / 1e9
    workload = f"{wl_key}: {G} x {R}-replica groups per GPU, {wl['desc']}, E={E}, K={K}"
    kname = ("tick_fused_kernel" if fuse > 1 else "tick_lean_kernel") if two_pass else "tick_fast_kernel"
    traffic, traffic_src = load_pmc(workload, kname, tpl)
    if traffic and fuse > 1:   # (the passes count bytes per launch, mean over launches; the roofline is per tick)
        traffic /= tpl
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "frac_measured": (traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
            "traffic_source": traffic_src,
            "bytes_per_group_step": B,
            "bytes_accounting": (("tick_fused_kernel, up to %d steady ticks per launch, %.4g on average over this "
                                  "call's launches (bench.py lean_bytes)" % (fuse, tpl)
                                  if fuse > 1 else
                                  "tick_lean_kernel, compressed steady state (bench.py lean_bytes), every group "
                                  "counted as taken by the lean pass") if two_pass else
                                 "SURVEY.md §8(d) B(R,E), per-replica SoA"),
            "ticks_per_launch": tpl,
            "max_ticks_per_launch": fuse,
            "units_per_launch": units,
            "kernel": ("tick_fused_kernel" if fuse > 1 else "tick_lean_kernel") if two_pass else "tick_fast_kernel",
            "avg_kernel_us": avg_kernel_s * 1e6, "kernel_launches": kernel_launches,
            "list_kernel_us": (list_ms * 1e3 / max(list_launches, 1)) if two_pass else None,
            "avg_region_us_per_tick": avg_region_s * 1e6,
            "achieved_region": B * units / avg_region_s / 1e9,
            # SURVEY §8(d)'s per-replica SoA figure at the measured tick rate:
            # the bandwidth an uncompressed SoA engine would need for this
            # throughput (above the HBM peak = beyond any per-replica layout)
            "survey_bytes_per_group_step": B_survey,
            "survey_equivalent_GBs": B_survey * value / world / 1e9}
    result = {
        "metric": "Raft group-steps/sec at 1M 5-replica groups, 1-8 GPUs; % of HBM peak",
        "value": value,
        "unit": "group-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded splitmix64 trace; %s, SURVEY.md §8(d) %s)"
                % ("NewNode start + isolation churn" if churn else "post-election steady state", wl_key),
        "config": {"workload": workload, "groups_per_gpu": G, "groups_total": G * world, "replicas": R,
                   "entries_per_tick": E, "ring_depth": K, "payload_crc32c": bool(crc), "leader": args.leader,
                   "seed": hex(wl["seed"]),
                   "semantics": "RAFT (EXT, Raft paper)" if wl.get("semantics") else "REF (main.go)",
                   "parallelism": f"group-sharded x{world}"},
        "timing": {"repeats": reps, "median_s": elapsed, "repeat_ms_per_step": [t * 1e3 / args.steps for t in times]},
        "roofline": roof,
        "stats": dict(zip(STAT_NAMES, [int(x) for x in stats])),
        "stats_check": bool(ok),
    }
    if wl.get("allow_faults"):   # REF prefix: groups frozen by a main.go panic / deadlock so far
        fi = STAT_NAMES.index("faults")
        result["faults_prefix"] = {"groups": G * world, "faulted_before_timed": int(untimed[fi]),
                                   "faulted_in_timed": int(stats[fi]),
                                   "frozen_fraction": (int(untimed[fi]) + int(stats[fi])) / (G * world),
                                   "value_counts": "live (not frozen) group-steps only",
                                   "live_group_steps_median_repeat": int(round(live_value * elapsed)),
                                   "all_group_steps_per_s": total_steps / elapsed}
    if world > 1:
        from raftstep import dist as rdist
        ranks = [None] * world
        dist.all_gather_object(ranks, {"rank": rank, "group_base": base, "groups": G, "rccl_nranks": nranks,
                                       "stat_allreduces": allreduces})
        result["multi_gpu"] = {"rccl_nranks": nranks if not same_dev else None,
                               "engine_communicator": not same_dev,
                               "per_rank": ranks}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, wl, R, E, K, crc)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if not ok:
        raise SystemExit("bench: statistics check failed")


if __name__ == "__main__":
    main()
