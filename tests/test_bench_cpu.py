"""CPU checks of bench.py's host logic (no GPU): the knob fence, the live
group-step count of the REF prefix line, the byte accounting."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_a_results_altering_knob():
    env = dict(os.environ, RAFTSTEP_DIAG_LEAN="64")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "RAFTSTEP_DIAG_LEAN" in r.stderr


def test_engine_env_records_every_raftstep_variable(monkeypatch):
    monkeypatch.setenv("RAFTSTEP_PIPELINE", "0")
    monkeypatch.setenv("RAFTSTEP_SOMETHING_ELSE", "1")
    env = bench.engine_env()
    assert env["RAFTSTEP_PIPELINE"]["value"] == "0" and env["RAFTSTEP_PIPELINE"]["effect"].startswith("exact")
    assert "unknown" in env["RAFTSTEP_SOMETHING_ELSE"]["effect"]
    assert all(k in bench.ENV_KNOBS for k in bench.RESULTS_ALTERING)


def test_live_group_steps_counts_each_group_step_once_over_ranks():
    """with an engine communicator the per-tick fault records are
    whole-job sums. Counting on the whole job's groups once gives the same
    live group-steps as counting each rank's own shard and summing; the
    round-3 formula (rank's groups minus whole-job faults, summed over ranks)
    subtracted the faults once per rank."""
    rng = np.random.default_rng(3)
    world, G, steps = 4, 1000, 20
    local = [rng.integers(0, 9, steps) for _ in range(world)]       # each rank's own faults per tick
    frozen_local = [int(x) for x in rng.integers(0, 50, world)]
    per_rank = sum(bench.live_group_steps(G, frozen_local[r], local[r]) for r in range(world))
    glob = bench.live_group_steps(G * world, sum(frozen_local), sum(local))
    assert per_rank == glob
    old = sum(G * steps - (sum(frozen_local) + np.concatenate([[0], np.cumsum(sum(local))[:-1]])).sum()
              for _ in range(world))
    assert old < glob
    assert glob <= G * world * steps


def test_live_group_steps_small_case():
    # 10 groups, 2 frozen before, 1 freezes during tick 0, 2 during tick 2
    assert bench.live_group_steps(10, 2, [1, 0, 2]) == 8 + 7 + 7


@pytest.mark.parametrize("R,E,crc,seg,fuse,glx,sh,want",
                         [(5, 1, 0, False, 1, False, False, 100), (7, 1, 0, True, 1, False, False, 128),
                          (7, 1, 0, True, 1, True, False, 136), (5, 64, 1, False, 1, False, False, 5160),
                          (5, 1, 0, False, 10, False, False, 64),
                          # shared entries (C2 / C5 / fused C2): one copy of each entry, no hb store
                          (5, 1, 0, False, 1, False, True, 48), (5, 64, 1, False, 1, False, True, 1060),
                          (5, 1, 0, False, 10, False, True, 15.6)])
def test_byte_accounting(R, E, crc, seg, fuse, glx, sh, want):
    assert bench.lean_bytes(R, E, crc, segmented=seg, fuse=fuse, glx=glx, shared=sh) == want


def test_survey_bytes():
    assert bench.algorithmic_bytes(5, 1) == 233 and bench.algorithmic_bytes(7, 1) == 331
    assert bench.algorithmic_bytes(5, 64, crc=True) == 5293


@pytest.mark.parametrize("name", ["C2", "C4"])
def test_cpu_leg_oracle_slice_check(name):
    """the CPU-baseline leg runs its oracle sample over a slice
    of the GPU line's groups through the same ticks and compares per-group
    digests. Here the 'engine' digests come from a full oracle of a small
    engine; one flipped digest inside the slice must fail the check."""
    import oracle
    wl = dict(bench.WORKLOADS[name], groups=3000)
    R = wl.get("replicas", bench.R_DEFAULT)
    kw = bench.engine_kwargs(wl, R, 3000, 0, wl["ring_depth"], wl["entries"], wl["crc"])
    full = oracle.Oracle(**kw)
    churn = wl.get("init") == "new"
    if churn:
        full.init_new_nodes(0)
        full.tick(0, wl["settle"] + 30)
        t_end = wl["settle"] + 30
    else:
        full.init_steady(0, 0)
        full.tick(1, 40)
        t_end = 41
    dig, _ = full.state_digest()
    full.close()
    cb = bench.cpu_baseline(wl, R, wl["entries"], wl["ring_depth"], wl["crc"], 1200, 64, check=(dig, t_end))
    sc = cb["oracle_slice_check"]
    assert sc["ok"] and sc["digests_differ"] == 0 and sc["digests_equal"] > 0, sc
    lo, hi = sc["groups"]
    assert 0 <= lo < hi <= 3000
    bad = dig.copy()
    bad[lo + (hi - lo) // 2] ^= 1
    sc2 = bench.cpu_baseline(wl, R, wl["entries"], wl["ring_depth"], wl["crc"], 1200, 64,
                             check=(bad, t_end))["oracle_slice_check"]
    assert not sc2["ok"] and sc2["digests_differ"] == 1
