"""Benchmark: Raft group-steps/sec (BASELINE.json metric) on MI355X.

One step = one tick of every group: client append of E
entries to the leader (main.go:327-329), one leader replication round to all
R-1 peers through their AppendEntries handlers (main.go:334-379, 121-156),
the commit rule (main.go:381-391) and the election timers. The headline
(`value`, `ms_per_step`, `roofline`) is measured in §8(d)'s form: ONE TICK PER
KERNEL LAUNCH (raft_config.ticks_per_launch = 1), every group's state read
from and written back to HBM every tick.

Workload at N=1: SURVEY config C2 — 2^20 independent 5-replica groups,
steady-state AppendEntries + commitIndex, one client entry per tick, seeded
synthetic trace. For N>1 the default is SURVEY config C3: each rank owns
2^21 groups (16M over 8 GPUs; weak scaling; groups shard by id, no
data-path collective); the per-tick statistics are reduced on the device and
summed across GPUs with RCCL on a side stream inside the engine.

Also in the same line (N=1, default workload):
  * `fused`: the same workload with up to 16 steady ticks per launch of
    tick_fused_kernel (ticks_per_launch = 16; state kept in registers between
    the ticks of a launch — NOT the §8(d) form, so never in `value` or
    `roofline`), with its own kernel fraction;
  * `extra_workloads`: SURVEY configs C4 (2^22 x 7 replicas, leader-isolation
    churn, RAFT semantics) and C5 (E=64 with CRC32C), each timed with the same
    protocol, with its own roofline and statistics check.

Protocol: W untimed warm-up ticks, then the timed region of
exactly K ticks (barrier + synchronize on both sides, max over ranks) is
repeated --repeats times (default 5) and the median is reported. The
roofline's `achieved` uses the dominant kernel's own average duration,
measured by HIP events attached to its dispatches on the engine stream
(profile mode 1) in a separate, untimed pass of K ticks: for the steady
lines one pair spanning the call's back-to-back launches (so it matches a
rocprofv3 kernel trace of the timed call), for the churn lines a pair on
every dispatch of the lean kernel.

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
FUSED_TICKS = 16        # ticks_per_launch of the `fused` block

# Environment knobs the engine reads (engine.cpp raft_engine_create). The
# bench records every RAFTSTEP_* variable it sees in config.engine_env and
# refuses to run with a results-altering one.
ENV_KNOBS = {
    "RAFTSTEP_DIAG_LEAN": "results-altering (timing diagnostics; the engine refuses it without debug_flags)",
    "RAFTSTEP_TWO_PASS": "exact: 0 = one-pass fast kernel (tests/test_gpu_parity.py)",
    "RAFTSTEP_FORCE_GENERAL": "exact: every group through the general kernel (tests/test_gpu_parity.py)",
    "RAFTSTEP_GENERAL": "exact: lane = one-lane-per-group general kernel (tests/test_gpu_tick_kat.py)",
    "RAFTSTEP_SLOW_EVERY": "exact: general-kernel window (tests/test_gpu_pipeline.py, test_gpu_dist.py)",
    "RAFTSTEP_PIPELINE": "exact: 0 = two passes in line (tests/test_gpu_pipeline.py)",
    "RAFTSTEP_PINGPONG": "exact: 0 = pipelined tick on a lean and a list stream instead of ping-pong streams "
                         "(tests/test_gpu_pipeline.py)",
    "RAFTSTEP_OVERLAP_GENERAL": "exact: 0 = general kernel in line, d = overlapping d ticks (tests/test_gpu_pipeline.py)",
    "RAFTSTEP_SPLIT_STEADY": "exact: 0 = one launch per steady tick instead of two halves on two streams "
                             "(tests/test_gpu_engine_checks.py)",
    "RAFTSTEP_SH": "exact: 0 = no shared entries (every entry in the R replica rings), 2 = shared entries under "
                   "isolation churn too (A/B only: 4x slower on C4; tests/test_gpu_sh.py)",
    "RAFTSTEP_VX": "exact: 0 = no virtual log suffixes (C4's stale leaders' entries stored and copied back at "
                   "their return; tests/test_gpu_fullsize.py, test_gpu_pipeline.py)",
    "RAFTSTEP_SH_KEEP": "exact: 0 = REF groups with corrupted copies leave the shared form (copied back) instead of "
                        "keeping it through the rejection (tests/test_gpu_sh.py)",
    "RAFTSTEP_SH_CHUNK": "exact: 0 = the shared ring one row per slot instead of 16-slot chunks where the list "
                         "kernel writes kept groups' batches (REF + corruption, E >= 16; tests/test_gpu_sh.py)",
    "RAFTSTEP_SHARD_SB": "exact: log2 of the consecutive 256-group blocks sharing a list / worklist shard chunk "
                         "(default: up to 64; 0 = the round-5 block-interleaved shards; A/B knob)",
    "RAFTSTEP_LIST_SORT": "exact: 0 = the list kernel ticks its staged groups in list order, not form order "
                          "(whole GPU suite with it on; an A/B knob)",
    "RAFTSTEP_LIST_BLOCKS": "exact: caps the list kernel's resident grid (A/B knob, round 6: the default grid was best)",
    "RAFTSTEP_DEBUG_WORK": "exact: prints worklist sizes, synchronises (in-line form)",
    "RAFTSTEP_DEBUG_PIPE": "exact: prints the pipeline choice",
    "RAFTSTEP_DEBUG_FAST": "exact: prints class counters after every call (synchronising)",
    "RAFTSTEP_LIB": "path of the library under test",
    "RAFTSTEP_BENCH_SAME_DEVICE": "test hook: N ranks on one GPU, gloo, no engine communicator",
    "RAFTSTEP_COMM_TIMEOUT_S": "exact: seconds raft_comm_init / a call's all-reduce may take before RAFT_ETIMEDOUT",
}
RESULTS_ALTERING = ("RAFTSTEP_DIAG_LEAN",)
TRAFFIC_SCOPE = ("memory-side bytes per launch (L2 egress: rocprofv3 FETCH_SIZE / WRITE_SIZE, calibrated), "
                 "Infinity-Cache (L3) hits included -- not HBM-only bytes")


def engine_env():
    """Every RAFTSTEP_* variable of this process, with what it does."""
    return {k: {"value": v, "effect": ENV_KNOBS.get(k, "unknown to this bench (not read by the engine)")}
            for k, v in sorted(os.environ.items()) if k.startswith("RAFTSTEP_")}


def algorithmic_bytes(R, E, crc=False):
    """minimal SoA bytes per group-step, REF steady state:
    B(R,E) = 25 + 37(R-1) + 12 E R (233 B at R=5, E=1; 331 B at R=7), + 4 E R
    with a CRC32C stamp per entry (C5: 5293 B). This is the per-replica SoA
    accounting (every replica's term/last/commit/deadline and every peer's
    MatchIndex read and written each tick); the compressed steady state
    needs less (lean_bytes), so the SURVEY figure is reported as an
    equivalent rate for the lean kernel and prices the list kernel's group-steps."""
    return 25 + 37 * (R - 1) + 12 * E * R + (4 * E * R if crc else 0)


def lean_bytes(R, E, crc=False, segmented=False, fuse=1, glx=False, shared=False, staged=False):
    """Algorithmic bytes per group-step of tick_lean_kernel (the dominant
    kernel of the two-pass tick, k_fast.hip) in this engine's layout: a group
    in the compressed steady state (SSYNC) holds term / LastApplied / the
    leader's and the followers' CommitIndex in one 16-B record, MatchIndex
    rows and follower timers are implicit (MSYNC, hb). Per group-step it
    reads gmeta 2 B + the record 16 B + the ring rotation 2 B (+ the ring
    segment boundary 4 B when the ring has 2K physical slots) and writes the
    record 16 B + hb 4 B + this tick's entries on all R replicas, 12 E R B
    (+4 E R with a CRC32C stamp). C2: 100 B; C4 shape (R=7, 2K slots): 128 B;
    C5: 5160 B. Under RAFT leader-isolation churn (`glx`) it also reads every
    group's 8-B glx word with the others (LXS / SXS state and HWX's mark, one
    round trip for every lane: k_fast.hip RAFTSTEP_LEAN_HOIST_LX): C4 136 B.
    With `fuse` ticks per launch (tick_fused_kernel, the `fused` block only)
    the record / meta / rotation / heartbeat bytes are moved once per launch:
    40 / fuse + 12 E R. With shared entries (`shared`, raft_engine_features:
    an in-step group's entries stored once, raft_device.hpp ROT_SH) the
    entries are written once instead of R times, 12 E (+4 E), and the
    heartbeat time is implied (DevPlanes::sh_hb: no hb store) — C2 48 B, C5
    1060 B. With staged client values (`staged`, RAFT_CLIENT_STAGED) it also
    reads the E values of the group's client request, 8 E B (SURVEY §8(d):
    "add 8E if client values are staged in HBM"): C2S 56 B, C4S 144 B."""
    copies = 1 if shared else R
    words = 20 + (4 if segmented else 0) + (8 if glx else 0) + 16 + (0 if shared else 4)
    return words / fuse + 12 * E * copies + (4 * E * copies if crc else 0) + (8 * E if staged else 0)


# SURVEY.md §8(d) workloads runnable by this bench (per GPU)
WORKLOADS = {
    "C2": dict(groups=1 << 20, entries=1, ring_depth=32, crc=0, seed=0x5EED0002,
               desc="steady-state AppendEntries+commit"),
    "C3": dict(groups=1 << 21, entries=1, ring_depth=32, crc=0, seed=0x5EED0003,
               desc="steady-state AppendEntries+commit, 2^21 groups per GPU (16M over 8 GPUs)"),
    # C2X: the C2 shape at 2^24 groups on one GPU, so that the
    # lean kernel's per-group words (40 B x 2^24 = 671 MB) cannot stay resident
    # in the 256 MiB Infinity Cache between ticks: its roofline fraction is the
    # HBM fraction (the 2^20 headline's bytes are partly L3-served)
    "C2X": dict(groups=1 << 24, entries=1, ring_depth=32, crc=0, seed=0x5EED0002,
                desc="steady-state AppendEntries+commit, C2 shape at 2^24 groups (beyond the Infinity Cache)"),
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
# Staged client values (raft_config.client_source = RAFT_CLIENT_STAGED,
# VERDICT r5 #1): the same workloads with every client value supplied by the
# caller in an HBM buffer (raft_stage_values, [ticks][E][G] int64) instead of
# the engine's trace RNG -- the drop-in LogReq path (main.go:87-93 ->
# 327-329). The engine cannot regenerate an entry in this mode (no virtual
# suffixes, no regenerated catch-up copies: those groups take the general
# kernel, which reads the leader's ring), and the lean kernel reads 8 B per
# group-step more. The values are staged before each timed region (inputs
# resident in HBM); `pcie_inclusive` times staging + ticks.
for _k in ("C2", "C4", "C5"):
    WORKLOADS[_k + "S"] = dict(WORKLOADS[_k], staged=True, desc=WORKLOADS[_k]["desc"] + ", client values staged by "
                               "the caller in HBM (RAFT_CLIENT_STAGED)")
# C5 with verification on the timed path: every follower's
# copy is corrupted w.p. 300/65536 per tick, so CRC32C rejections (and the
# backoff of the rejecting followers) happen inside the timed region
# (K = 512: a follower that rejected j batches in a row is sent (j+1) x 64
# entries with prevLogIndex j x 64 + 64 back; REF faults with RING_EVICTED
# once that leaves the window, i.e. after 7 rejections in a row here, after
# one with C5's K = 128)
WORKLOADS["C5V"] = dict(WORKLOADS["C5"], corrupt=300, ring_depth=512,
                        desc=WORKLOADS["C5"]["desc"] + ", EXT corruption 300/65536 per follower and tick (rejections "
                                                       "timed)")
EXTRA_DEFAULT = ("C2X", "C4", "C5", "C2S", "C4S", "C5V")


def _sm64_np(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


_KEYS = {}   # staged_values: the per-group keys of the last (seed, base, groups)


def staged_values(seed, group_base, groups, first_tick, nticks, E):
    """The client's values for RAFT_CLIENT_STAGED lines and tests: [nticks][E][G]
    int64 in [0, 2^63) like rand.Int() (main.go:92), a hash of (seed, global
    group id, tick, entry) made by the CALLER (numpy, independent of the
    engine's trace RNG), so that any slice of groups can be re-staged for an
    oracle slice: a hashed per-group key XOR a hashed (tick, entry) word, one
    pass per value (staging 2^22 groups x 20 ticks takes well under a second)."""
    with np.errstate(over="ignore"):
        ck = (seed, group_base, groups)
        key = _KEYS.get(ck)
        if key is None:
            gid = np.arange(group_base, group_base + groups, dtype=np.uint64)
            key = _sm64_np(gid ^ np.uint64(seed ^ 0xC11E57A6ED)) >> np.uint64(1)
            _KEYS.clear()
            _KEYS[ck] = key
        q = np.arange(first_tick, first_tick + nticks, dtype=np.uint64)[:, None] * np.uint64(E) + \
            np.arange(E, dtype=np.uint64)[None, :]
        q = _sm64_np(q ^ np.uint64(seed)) >> np.uint64(1)
        return (key[None, None, :] ^ q[:, :, None]).view(np.int64)


def cpu_baseline(wl, R, E, K, crc, groups, ticks, leader=0, check=None):
    """The oracle (C restatement of main.go's handlers, oracle/) timed on the
    host cores on a bounded sample of the same workload: G groups (scaled
    down) started at global offset `off`, run from the same start state
    through the same ticks as the GPU engine (the trace RNG is keyed by the
    global group id and groups never address each other, main.go:12, 259,
    334, so the sample evolves exactly like those groups inside the engine).

    check = (engine per-group digests, engine's next tick): the sample is run
    at least up to the tick the engine stopped at, and there (outside the
    timed span) its per-group digests are compared with the engine's digests
    of the same groups -- the line's oracle check (a
    wrong-but-plausible kernel cannot produce a line). The checker is the
    oracle only here, in the CPU-baseline leg; the engine never calls it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    G, T = groups, ticks
    if E > 1:   # keep the sample's CPU time and memory bounded for big batches
        G, T = max(1024, 4 * G // E), max(16, T // 4)
    Geng = wl["groups"] if check is None else len(check[0])
    G = min(G, Geng)
    # a seeded, unaligned offset inside the engine's group range
    off = 0 if G >= Geng else int(np.random.default_rng(wl["seed"]).integers(0, Geng - G + 1))
    staged = bool(wl.get("staged"))

    def stage(o, t, n):   # RAFT_CLIENT_STAGED: the slice's columns of the line's values (untimed)
        if staged and n > 0:
            o.stage_values(t, staged_values(wl["seed"], off, G, t, n, E))

    if wl.get("init") == "new":
        G, T = max(1, G // 2), max(1, T // 2)
        o = oracle.Oracle(**engine_kwargs(wl, R, G, off, K, E, crc))
        o.init_new_nodes(0)
        stage(o, 0, wl["settle"])
        o.tick(0, wl["settle"], threads=threads)
        t_first, start = wl["settle"], "after a NewNode start and %d settle ticks" % wl["settle"]
    else:
        o = oracle.Oracle(**engine_kwargs(wl, R, G, off, K, E, crc))
        o.init_steady(leader, 0)
        t_first, start = 1, "steady state from init_steady"
    slice_check = None
    dt = 0.0
    t = t_first
    if check is not None:
        dig, t_end = check
        T = max(T, t_end - t_first)
        stage(o, t, t_end - t)
        t0 = time.perf_counter()
        o.tick(t, t_end - t, threads=threads)
        dt += time.perf_counter() - t0
        t = t_end
        do, _ = o.state_digest()
        bad = np.nonzero(np.asarray(dig[off:off + G]) != do)[0]
        slice_check = {"groups": [off, off + G], "ticks": [0 if wl.get("init") == "new" else 1, t_end],
                       "digests_equal": int(G - bad.size), "digests_differ": int(bad.size),
                       "first_bad_group": (off + int(bad[0])) if bad.size else None, "ok": not bad.size,
                       "what": "per-group state digests (raft_state_digest) of the GPU engine after the line's "
                               "last call vs the oracle run over the same groups and ticks"}
    rest = t_first + T - t
    if rest > 0:
        stage(o, t, rest)
        t0 = time.perf_counter()
        o.tick(t, rest, threads=threads)
        dt += time.perf_counter() - t0
    o.close()
    out = {"value": G * T / dt, "unit": "group-steps/s", "cores": threads, "kind": "port",
           "sample": f"{G} groups [{off}, {off + G}) of the GPU line's {Geng} x {T} ticks, R={R}, E={E}, "
                     f"crc={crc}, {start}; oracle/raft_oracle.c (C restatement of main.go's handlers), "
                     f"{threads} pthreads over contiguous group ranges ({dt:.2f} s)"}
    if slice_check is not None:
        out["oracle_slice_check"] = slice_check
    return out


def engine_kwargs(wl, R, G, base, K, E, crc):
    kw = dict(replicas=R, groups=G, group_base=base, ring_depth=K, entries_per_tick=E, client_period=1,
              payload_crc=crc, seed=wl["seed"], semantics=wl.get("semantics", 0),
              client_source=1 if wl.get("staged") else 0, corrupt_per_65536=wl.get("corrupt", 0))
    if "iso" in wl:
        kw.update(isolate_per_65536=wl["iso"][0], isolate_min_ticks=wl["iso"][1], isolate_max_ticks=wl["iso"][2],
                  isolate_leader=wl["iso"][3])
    return kw


def load_pmc(workload, kernel, ticks=1):
    """HBM traffic per launch of a kernel from the committed rocprofv3 --pmc
    summary of exactly this workload, kernel and ticks per launch (mean over
    the pass's launches; profiles/pmc_*.json, made by tools/pmc_summary.py
    from FETCH_SIZE / WRITE_SIZE passes), and where it came from; (None,
    None) if no pass covers it."""
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
            return d, src
    return None, None


def live_group_steps(groups, frozen, faults_per_tick):
    """Group-steps of the groups not frozen by a fault (REF prefix, C4REF):
    `groups` groups, `frozen` of them frozen before the first tick, and
    faults_per_tick[t] groups freezing during tick t (a group that faults
    during a tick did that tick's work). All three must count the same scope:
    with the engine's RCCL communicator the per-tick records are already
    summed over every rank, so `groups` is then the whole job's (ADVICE r3:
    subtracting whole-job fault counts from one rank's groups, then summing
    over ranks, subtracted them once per rank)."""
    f = np.asarray(faults_per_tick, np.int64)
    before = frozen + np.concatenate([[0], np.cumsum(f)[:-1]])
    return int(groups * len(f) - before.sum())


def median(xs):
    xs = sorted(xs)
    n = len(xs)
    return xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])


class Ctx:
    """Process / rank context of one bench run."""

    def __init__(self, world, rank, local, dist, same_dev):
        self.world, self.rank, self.local, self.dist, self.same_dev = world, rank, local, dist, same_dev

    @property
    def comm(self):   # the engine carries an RCCL communicator over every rank
        return self.dist is not None and not self.same_dev

    def barrier(self):
        import torch
        torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()
        torch.cuda.synchronize()


def measure(ctx, wl_key, wl, G, R, E, K, steps, warmup, repeats, tpl=1, leader=0, cpu=None, list_count=True):
    """One line: `repeats` timed regions of exactly `steps` ticks of workload
    `wl` on this rank's shard (G groups) with `tpl` ticks per launch, then the
    untimed profile passes for the dominant kernel's duration. Returns the
    line's fields (value over all ranks)."""
    from raftstep import Engine, STAT_NAMES
    from raftstep import dist as rdist
    world, dist = ctx.world, ctx.dist
    crc = wl["crc"]
    churn = wl.get("init") == "new"
    base = ctx.rank * G
    eng = Engine(device=ctx.local, ticks_per_launch=tpl, **engine_kwargs(wl, R, G, base, K, E, crc))
    feats = eng.features()
    shared = feats["shared_entries"]
    if ctx.comm:
        eng.comm_init(world, ctx.rank, rdist.exchange_comm_id(dist, ctx.rank, Engine.comm_unique_id))
    fi = STAT_NAMES.index("faults")
    staged = bool(wl.get("staged"))

    def stage(t, n):   # RAFT_CLIENT_STAGED: the caller's values for ticks [t, t+n) into HBM (never timed)
        if staged and n > 0:
            eng.stage_values(t, staged_values(wl["seed"], base, G, t, n, E))

    untimed = np.zeros(len(STAT_NAMES), np.int64)   # stats of the settle and warm-up ticks
    if churn:   # NewNode start; the first elections happen in untimed settle ticks
        eng.init_new_nodes(0)
        stage(0, wl["settle"])
        untimed += eng.tick(0, wl["settle"], stats=True)
        tick = wl["settle"]
    else:
        eng.init_steady(leader, 0)
        tick = 1
    if warmup:
        stage(tick, warmup)
        untimed += eng.tick(tick, warmup, stats=True)
        tick += warmup

    # timed regions: exactly `steps` ticks each (+ the per-tick stats, reduced
    # on the device and, at N>1, all-reduced by RCCL on the engine's side stream)
    times, stats = [], np.zeros(len(STAT_NAMES), np.int64)
    local_times = []   # this rank's own wall time per repeat (multi_gpu.per_rank)
    # C4REF (REF prefix): a group frozen by a fault does no work, so the value
    # counts only the live group-steps. With the engine communicator every
    # record is already the sum over all ranks, so the live count is computed
    # once over the whole job; without one each rank counts its own shard.
    scope = G * world if ctx.comm else G
    frozen = int(untimed[fi])
    live_steps = []
    for _ in range(max(1, repeats)):
        stage(tick, steps)   # (inputs resident in HBM before the timed region)
        ctx.barrier()
        t0 = time.perf_counter()
        s = eng.tick(tick, steps, stats=True)
        ctx.barrier()
        el = time.perf_counter() - t0
        local_times.append(el)
        if wl.get("allow_faults"):   # (outside the timed region) per-tick fault counts
            f = eng.tick_records(steps)[:, fi]
            live_steps.append(live_group_steps(scope, frozen, f))
            frozen += int(f.sum())
        if dist is not None:
            el = rdist.max_over_ranks(dist, el, device=None if ctx.same_dev else "cuda")
            if ctx.same_dev:   # no engine communicator: sum the stats through torch.distributed
                s = np.array(rdist.sum_over_ranks(dist, s), np.int64)
        times.append(el)
        stats += s
        tick += steps
    # untimed passes: the steady-state kernel's own duration (events attached
    # to each of its dispatches), then the list kernel's and its group-steps
    two_pass = os.environ.get("RAFTSTEP_TWO_PASS", "1") != "0"
    pcie = None
    if staged:
        # the same call with the values crossing PCIe inside the timed span
        # (raft_stage_values from host memory, then the ticks): never `value`
        vals = staged_values(wl["seed"], base, G, tick, steps, E)
        ctx.barrier()
        t0 = time.perf_counter()
        eng.stage_values(tick, vals)
        t1 = time.perf_counter()
        eng.tick(tick, steps, stats=True)
        ctx.barrier()
        t2 = time.perf_counter()
        tick += steps
        pcie = {"value": G * world * steps / (t2 - t0), "stage_ms": (t1 - t0) * 1e3,
                "stage_GBs": vals.nbytes / max(t1 - t0, 1e-9) / 1e9, "ms_per_step": (t2 - t0) * 1e3 / steps,
                "what": "raft_stage_values (host buffer -> HBM, %d MB) + the %d ticks, one call, wall clock"
                        % (vals.nbytes // 1000000, steps)}
        del vals
    eng.profile(1)
    stage(tick, steps)
    eng.tick(tick, steps, stats=False)
    tick += steps
    kernel_ms, kernel_ticks = eng.profile_read()
    list_ms = list_launches = list_steps = 0
    if two_pass and churn:   # the second pass (list kernel over the groups the lean kernel passed on)
        eng.profile(3)
        stage(tick, steps)
        eng.tick(tick, steps, stats=False)
        tick += steps
        list_ms, list_launches = eng.profile_read()
        eng.profile(0)
        if list_count:   # (separately: the class counters cost time) listed group-steps per launch
            eng.diag_enable(True)
            stage(tick, steps)
            eng.tick(tick, steps, stats=False)
            tick += steps
            list_steps = eng.diag_read()["list_lanes"]
            eng.diag_enable(False)
    eng.profile(0)
    nranks, _, allreduces = eng.comm_info()
    do_cpu = cpu and ctx.rank == 0 and world == 1
    digests = eng.state_digest()[0] if do_cpu else None   # (the CPU leg's oracle check, untimed)
    eng.close()

    reps = len(times)
    elapsed = median(times)
    total_steps = G * world * steps
    value = total_steps / elapsed
    live_value = None
    if wl.get("allow_faults"):
        mid = sorted(range(reps), key=lambda i: times[i])[reps // 2]
        live = live_steps[mid]
        if dist is not None and not ctx.comm:
            live = int(sum(rdist.sum_over_ranks(dist, [live])))
        live_value = live / times[mid]
        value = live_value
    # correctness guard on the timed runs: the steady state commits exactly one
    # entry per group per tick and never faults; under churn nothing faults
    # and most groups have a leader (REF prefix: faults are the point)
    faults = int(stats[fi])
    if churn:
        ok = bool(wl.get("allow_faults") or
                  (faults == 0 and stats[STAT_NAMES.index("leader_groups")] > 0.5 * G * world * steps * reps))
    elif wl.get("corrupt"):
        # CRC32C rejections in the timed region: a rejected copy fails that
        # follower's AppendEntries (the only failures of a steady REF group);
        # the leader still commits whenever 3 of its 4 peers match
        ok = bool(faults * 100000 <= G * world and stats[STAT_NAMES.index("ae_fail")] > 0 and
                  stats[STAT_NAMES.index("committed")] > 0.99 * G * world * steps * E * reps)
    else:
        ok = bool(stats[STAT_NAMES.index("committed")] == G * world * steps * E * reps and faults == 0)

    # roofline of the dominant kernel, in its own layout's algorithmic bytes:
    # the lean kernel (one tick per launch) or the fused kernel (tpl > 1,
    # priced at the call's mean ticks per launch: K = 20 at 16 is 16 + 4)
    fused = tpl > 1 and not churn and not crc and two_pass
    mean_tpl = steps / -(-steps // tpl) if fused else 1
    iso = "iso" in wl and wl["iso"][0] > 0
    # (2K physical ring slots, whose segment boundary the lean kernel reads: under
    # isolation churn and, round 6, with corrupted copies — DevPlanes::sh_keep)
    B = lean_bytes(R, E, crc, segmented=iso or bool(crc and wl.get("corrupt")), fuse=mean_tpl,
                   glx=iso and wl.get("semantics", 0) == 1,
                   shared=shared, staged=staged) if two_pass else \
        algorithmic_bytes(R, E, crc) + (8 * E if staged else 0)
    kname = ("tick_fused_kernel" if fused else "tick_lean_kernel") if two_pass else "tick_fast_kernel"
    avg_kernel_s = kernel_ms / 1e3 / max(kernel_ticks, 1)   # per tick
    # C4REF: the lean kernel's algorithmic bytes are those of the live groups it
    # takes (a frozen group is read as 2 B of gmeta and skipped)
    units = G if live_value is None else live_value * elapsed / world / steps
    achieved = B * units / avg_kernel_s / 1e9
    workload = f"{wl_key}: {G} x {R}-replica groups per GPU, {wl['desc']}, E={E}, K={K}"
    pmc, pmc_src = load_pmc(workload, kname, mean_tpl)
    # per tick (a steady tick is two launches over the halves of the groups)
    traffic = (pmc.get("hbm_bytes_per_tick") or pmc["hbm_bytes_per_launch"]) / mean_tpl if pmc else None
    B_survey = algorithmic_bytes(R, E, crc)
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_scope": TRAFFIC_SCOPE,
            "frac_measured": (traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
            "traffic_source": pmc_src,
            "kernel": kname,
            "ticks_per_launch": mean_tpl,
            "max_ticks_per_launch": tpl if fused else 1,
            "bytes_per_group_step": B,
            "bytes_accounting": (
                ("tick_fused_kernel, up to %d steady ticks per launch, %.4g on average over this call's launches "
                 "(bench.py lean_bytes; NOT SURVEY §8(d)'s one-tick-per-launch form)" % (tpl, mean_tpl))
                if fused else
                ("tick_lean_kernel, one tick per launch, compressed steady state (bench.py lean_bytes), every "
                 "group counted as taken by the lean pass; steady lines: the tick's launches (two halves of the "
                 "groups on two streams) timed as one span per call" +
                 ("; shared entries (each entry stored once for the R replicas that hold it alike)"
                  if shared else "")) if two_pass else
                "SURVEY.md §8(d) B(R,E), per-replica SoA"),
            "units_per_launch": units * (mean_tpl if fused else 1),
            "avg_kernel_us": avg_kernel_s * 1e6 * (mean_tpl if fused else 1),
            "avg_kernel_us_per_tick": avg_kernel_s * 1e6,
            # the same bytes over the timed region's wall clock (host launch
            # and readback included): a profiler-free lower bound of `achieved`
            "achieved_wall": B * value / world / 1e9,
            "frac_wall": B * value / world / 1e9 / HBM_PEAK_GBS,
            "kernel_launches": kernel_ticks if not fused else -(-kernel_ticks // tpl),
            # SURVEY §8(d)'s per-replica SoA figure at the measured tick rate:
            # the bandwidth an uncompressed SoA engine would need for this
            # throughput (above the HBM peak = beyond any per-replica layout)
            "survey_bytes_per_group_step": B_survey,
            "survey_equivalent_GBs": B_survey * value / world / 1e9}
    line = {
        "value": value, "ms_per_step": elapsed * 1e3 / steps, "steps": steps, "warmup": warmup,
        "workload": workload, "groups_per_gpu": G, "groups_total": G * world, "replicas": R,
        "entries_per_tick": E, "ring_depth": K, "payload_crc32c": bool(crc), "seed": hex(wl["seed"]),
        "semantics": "RAFT (EXT, Raft paper)" if wl.get("semantics") else "REF (main.go)",
        "ticks_per_launch": tpl,
        "storage_forms": feats,
        "client_values": ("staged by the caller in HBM (RAFT_CLIENT_STAGED, raft_stage_values), never regenerated"
                          if staged else "trace RNG on the device (RAFT_CLIENT_TRACE)"),
        "timing": {"repeats": reps, "median_s": elapsed, "repeat_ms_per_step": [t * 1e3 / steps for t in times]},
        "roofline": roof,
        "stats": dict(zip(STAT_NAMES, [int(x) for x in stats])),
        "stats_check": ok,
        "rccl": {"nranks": nranks, "stat_allreduces": allreduces},
    }
    if pcie is not None:
        line["pcie_inclusive"] = pcie
    if wl.get("corrupt"):
        st = line["stats"]
        line["verification"] = {
            "corrupt_per_65536": wl["corrupt"], "rejections": st["ae_fail"],
            "entries_verified": (st["ae_ok"] + st["ae_fail"]) * E,
            "what": "every follower checks each received entry against the leader's CRC32C stamp (an unaltered "
                    "copy carries the stamp itself; a corrupted copy -- its last value's bit 0 flipped -- is "
                    "recomputed and rejected: AppendEntries false, main.go:148-149 append skipped); rejections = "
                    "AppendEntries answered false in the timed region"}
    if two_pass and churn:
        # the list kernel: the full fast-path body over the groups the lean
        # kernel passed on (elections, first rounds, returns, isolated
        # leaders), two steps per launch in the pipelined tick, priced with
        # SURVEY §8(d)'s per-replica bytes per group-step it advances
        lus = list_ms * 1e3 / max(list_launches, 1)
        per_launch = list_steps / max(list_launches, 1)
        lpmc, lsrc = load_pmc(workload, "tick_list_kernel", 1)
        line["list_kernel"] = {
            "avg_us": lus, "launches": list_launches, "group_steps_per_launch": per_launch,
            "bytes_per_group_step": B_survey,
            "achieved": B_survey * per_launch / max(lus, 1e-9) / 1e3, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": B_survey * per_launch / max(lus, 1e-9) / 1e3 / HBM_PEAK_GBS,
            "traffic_per_group_step": (lpmc["hbm_bytes_per_launch"] / per_launch) if (lpmc and per_launch) else None,
            "traffic_source": lsrc}
    if wl.get("allow_faults"):   # REF prefix: groups frozen by a main.go panic / deadlock so far
        uf = int(untimed[fi])   # (with the engine communicator already the sum over ranks)
        if dist is not None and not ctx.comm:
            uf = int(sum(rdist.sum_over_ranks(dist, [uf])))
        line["faults_prefix"] = {"groups": G * world, "faulted_before_timed": uf, "faulted_in_timed": faults,
                                 "frozen_fraction": (uf + faults) / (G * world),
                                 "value_counts": "live (not frozen) group-steps only",
                                 "live_group_steps_median_repeat": int(round(live_value * elapsed)),
                                 "all_group_steps_per_s": total_steps / elapsed}
    # this rank's own numbers (multi_gpu.per_rank: where scaling is lost)
    line["rank_local"] = {"ms_per_step": median(local_times) * 1e3 / steps,
                          "repeat_ms_per_step": [x * 1e3 / steps for x in local_times],
                          "lean_kernel_us_per_tick": avg_kernel_s * 1e6, "stat_allreduces": allreduces}
    if world == 1 and not churn and not crc and E == 1 and not fused and hasattr(eng.lib, "raft_stream_probe"):
        # this device's sustained rate for the lean kernel's byte mix and access
        # shape at the same size (raft_stream_probe: fresh buffers, no Raft
        # state): the practical roofline of this kernel on this box
        from raftstep import stream_probe
        # (shared entries: the probe's ring row is one copy wide, R=1, and it
        # skips the heartbeat store as the kernel does: 48 B)
        pus, pby = stream_probe(ctx.local, 1 if shared else R, G, 10, heartbeat=not shared)
        pb = (36 if shared else 40) + 12 * (1 if shared else R)
        roof["stream_probe"] = {"GBs": pby / pus / 1e3, "us_per_pass": pus, "bytes_per_pass": pby,
                                "what": "raft_stream_probe: per element 20 B read in one round trip, %d B moved "
                                        "(%d ring copies%s), record%s / whole-ring-row stores, on fresh buffers of "
                                        "the line's group count"
                                        % (pb, 1 if shared else R, ", no heartbeat store" if shared else "",
                                           "" if shared else " / heartbeat")}
        roof["frac_of_stream_probe"] = achieved / (pby / pus / 1e3)
    if do_cpu:
        cb = cpu_baseline(wl, R, E, K, crc, *cpu, leader=leader, check=(digests, tick))
        line["cpu_baseline"] = cb
        sc = cb.get("oracle_slice_check")
        if sc is not None:
            line["oracle_slice_check"] = sc
            line["stats_check"] = bool(line["stats_check"] and sc["ok"])
    return line


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
    ap.add_argument("--no-fused", action="store_true", help="skip the `fused` block")
    ap.add_argument("--extra", default=None,
                    help="comma-separated extra workloads timed after the headline at N=1 (default C4,C5 with the "
                         "default workload; 'none' to skip)")
    ap.add_argument("--extra-budget", type=float, default=120.0,
                    help="seconds: no further extra workload starts once the run has taken this long")
    ap.add_argument("--no-list-count", action="store_true",
                    help="skip the untimed pass that counts the list kernel's group-steps with the class counters "
                         "(its atomics make that pass slow; profiler runs leave it out)")
    ap.add_argument("--isolate", type=int, default=None,
                    help="diagnostics: override the workload's isolation windows per 65536 epochs (0: none)")
    args = ap.parse_args()
    t_start = time.perf_counter()

    env = engine_env()
    bad = [k for k in env if k in RESULTS_ALTERING]
    if bad:
        raise SystemExit(f"bench: {bad} alter results; refusing to time with them")

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
        import datetime
        import torch.distributed as dist
        torch.cuda.set_device(local)
        # a rank that never arrives ends the run with an error, not a hang
        # (the engine's own communicator is bounded the same way, raftstep.h)
        tmo = datetime.timedelta(seconds=float(os.environ.get("RAFTSTEP_COMM_TIMEOUT_S", "300")))
        if same_dev:
            dist.init_process_group("gloo", timeout=tmo)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
    ctx = Ctx(world, rank, local, dist, same_dev)

    wl = WORKLOADS[wl_key]
    if args.isolate is not None and "iso" in wl:
        wl = dict(wl, iso=(args.isolate,) + tuple(wl["iso"][1:]))
    R = args.replicas or wl.get("replicas", R_DEFAULT)
    G = args.groups_per_gpu or wl["groups"]
    E = args.entries or wl["entries"]
    K = args.ring_depth or wl["ring_depth"]
    cpu = None if args.no_cpu_baseline else (args.cpu_groups, args.cpu_ticks)
    head = measure(ctx, wl_key, wl, G, R, E, K, args.steps, args.warmup, args.repeats, tpl=1, leader=args.leader,
                   cpu=cpu, list_count=not args.no_list_count)
    ok = head["stats_check"]

    multi = None
    if world > 1:
        ranks = [None] * world
        rl = head["rank_local"]
        dist.all_gather_object(ranks, {"rank": rank, "group_base": rank * G, "groups": G,
                                       "rccl_nranks": head["rccl"]["nranks"],
                                       "stat_allreduces": head["rccl"]["stat_allreduces"],
                                       "ms_per_step": rl["ms_per_step"],
                                       "repeat_ms_per_step": rl["repeat_ms_per_step"],
                                       "lean_kernel_us_per_tick": rl["lean_kernel_us_per_tick"]})
        multi = {"rccl_nranks": head["rccl"]["nranks"] if not same_dev else None,
                 "engine_communicator": not same_dev, "per_rank": ranks}
        if not same_dev:
            # the engine communicator must span every rank, and every window's
            # stats must have gone through it (ncclAllReduce on the side stream)
            if any(r["rccl_nranks"] != world for r in ranks):
                raise SystemExit(f"bench: RCCL communicator ranks {[r['rccl_nranks'] for r in ranks]}, "
                                 f"WORLD_SIZE is {world}")
            ok = ok and all(r["stat_allreduces"] > 0 for r in ranks)

    steady_default = args.workload is None and world == 1 and not any(
        x is not None for x in (args.groups_per_gpu, args.replicas, args.entries, args.ring_depth))
    fused = None
    if world == 1 and not args.no_fused and wl.get("init") != "new" and not wl["crc"]:
        fl = measure(ctx, wl_key, wl, G, R, E, K, args.steps, args.warmup, args.repeats, tpl=FUSED_TICKS,
                     leader=args.leader)
        ok = ok and fl["stats_check"]
        fused = {"note": "NOT the headline: up to %d steady ticks per launch of tick_fused_kernel, state kept in "
                         "registers between the ticks of a launch (SURVEY §8(d) excludes this form from the "
                         "roofline claim); same workload, protocol and statistics check" % FUSED_TICKS,
                 "value": fl["value"], "ms_per_step": fl["ms_per_step"], "ticks_per_launch": FUSED_TICKS,
                 "roofline": fl["roofline"], "stats_check": fl["stats_check"],
                 "timing": fl["timing"]}

    extras = {}
    names = EXTRA_DEFAULT if (args.extra is None and steady_default) else \
        tuple(x for x in (args.extra or "").split(",") if x and x != "none")
    if world > 1:
        names = ()
    for name in names:
        if time.perf_counter() - t_start > args.extra_budget:
            extras[name] = {"skipped": f"extra budget of {args.extra_budget:.0f} s spent"}
            continue
        xw = WORKLOADS[name]
        xR, xE, xK = xw.get("replicas", R_DEFAULT), xw["entries"], xw["ring_depth"]
        x = measure(ctx, name, xw, xw["groups"], xR, xE, xK, args.steps, args.warmup, args.repeats, tpl=1,
                    cpu=None if args.no_cpu_baseline else (args.cpu_groups // 4, args.cpu_ticks // 4),
                    list_count=not args.no_list_count)
        ok = ok and x["stats_check"]
        x.pop("rccl", None)
        extras[name] = x

    result = {
        "metric": "Raft group-steps/sec at 1M 5-replica groups, 1-8 GPUs; % of HBM peak",
        "value": head["value"],
        "unit": "group-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded splitmix64 trace; %s, SURVEY.md §8(d) %s)"
                % ("NewNode start + isolation churn" if wl.get("init") == "new" else "post-election steady state",
                   wl_key),
        "config": {"workload": head["workload"], "groups_per_gpu": G, "groups_total": G * world, "replicas": R,
                   "entries_per_tick": E, "ring_depth": K, "payload_crc32c": bool(wl["crc"]), "leader": args.leader,
                   "seed": hex(wl["seed"]), "semantics": head["semantics"],
                   "ticks_per_launch": 1, "parallelism": f"group-sharded x{world}", "engine_env": env},
        "timing": head["timing"],
        "roofline": head["roofline"],
        "stats": head["stats"],
        "stats_check": bool(ok),
    }
    for k in ("list_kernel", "faults_prefix"):
        if k in head:
            result[k] = head[k]
    if multi:
        result["multi_gpu"] = multi
    if rank == 0:
        result["cpu_baseline"] = head.get("cpu_baseline")
    if fused:
        result["fused"] = fused
    if extras:
        result["extra_workloads"] = extras
        x = extras.get("C2X")
        if x and "roofline" in x:
            # the HBM fraction proper: the same kernel and bytes per group-step
            # at a size whose per-group words cannot stay in the Infinity Cache
            xr = x["roofline"]
            result["roofline"]["l3_proof"] = {
                "workload": x["workload"], "groups": x["groups_per_gpu"], "achieved": xr["achieved"],
                "frac": xr["frac"], "frac_wall": xr["frac_wall"], "avg_kernel_us_per_tick": xr["avg_kernel_us_per_tick"],
                "stream_probe_GBs": (xr.get("stream_probe") or {}).get("GBs"),
                "frac_of_stream_probe": xr.get("frac_of_stream_probe"),
                "per_group_words_MB": 40 * x["groups_per_gpu"] / 1e6, "infinity_cache_MB": 256 * 1.048576,
                "note": "the headline's 2^20 groups keep their 40 B of per-group words (42 MB) L3-resident between "
                        "ticks, so part of its `achieved` is Infinity-Cache-served; this line's frac is the HBM "
                        "fraction of the same kernel (extra_workloads.C2X)"}
    # flat copies of the nested numbers a reader of the driver's record needs
    # (the driver's `parsed` keeps top-level scalars only)
    r0 = result["roofline"]
    flat = {"roofline_frac": r0["frac"], "roofline_achieved_GBs": r0["achieved"],
            "lean_kernel_us_per_tick": r0["avg_kernel_us_per_tick"],
            "stream_probe_GBs": (r0.get("stream_probe") or {}).get("GBs"),
            "frac_of_stream_probe": r0.get("frac_of_stream_probe"),
            "l3_proof_frac": (r0.get("l3_proof") or {}).get("frac"),
            "l3_proof_GBs": (r0.get("l3_proof") or {}).get("achieved"),
            "cpu_baseline_value": (result.get("cpu_baseline") or {}).get("value"),
            "fused_value": (fused or {}).get("value")}
    for name, x in extras.items():
        if "value" not in x:
            continue
        flat[f"{name}_value"] = x["value"]
        flat[f"{name}_frac"] = x["roofline"]["frac"]
        flat[f"{name}_kernel_us"] = x["roofline"]["avg_kernel_us_per_tick"]
        flat[f"{name}_stats_check"] = x["stats_check"]
        if "pcie_inclusive" in x:
            flat[f"{name}_pcie_inclusive_value"] = x["pcie_inclusive"]["value"]
        if "verification" in x:
            flat[f"{name}_rejections"] = x["verification"]["rejections"]
        if "list_kernel" in x:
            flat[f"{name}_list_kernel_us"] = x["list_kernel"]["avg_us"]
    result["flat"] = "the *_value / *_frac / ... keys below copy nested numbers to the top level"
    result.update({k: v for k, v in flat.items() if v is not None})
    result["bench_wall_s"] = time.perf_counter() - t_start
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if not ok:
        raise SystemExit("bench: statistics check failed")


if __name__ == "__main__":
    main()
