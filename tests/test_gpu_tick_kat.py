"""GPU: the engine through raft_tick against the hand-derived tick-level
KATs of kat_tick.py, on every device path: the steady-state kernel with the
replica-parallel general kernel behind it (auto), every group forced through
the general kernel, and the one-lane-per-group general kernel."""
import pytest

import kat_tick
from raftstep import Engine

pytestmark = pytest.mark.gpu

PATHS = {"auto": {"RAFTSTEP_FORCE_GENERAL": "0"},
         "single": {"RAFTSTEP_FORCE_GENERAL": "0", "RAFTSTEP_TWO_PASS": "0"},
         "general": {"RAFTSTEP_FORCE_GENERAL": "1"},
         "general_lane": {"RAFTSTEP_FORCE_GENERAL": "1", "RAFTSTEP_GENERAL": "lane"}}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("name", sorted(kat_tick.CASES))
def test_engine_tick_kat(monkeypatch, name, path):
    for k, v in PATHS[path].items():
        monkeypatch.setenv(k, v)
    for slow_every in ("1", "8"):
        monkeypatch.setenv("RAFTSTEP_SLOW_EVERY", slow_every)
        kat_tick.run_case(Engine, name)
