"""CPU: the oracle through whole ticks against the hand-derived tick-level
KATs of kat_tick.py (main.go text + the documented tick model), and the
test's own restatement of the trace RNG against the committed vectors."""
import json
import os

import pytest

import kat_tick
import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_trace_rng_restatement_matches_vectors():
    for v in json.load(open(os.path.join(GOLDEN, "rng_vectors.json"))):
        assert kat_tick.trace_rng(v["seed"], v["gid"], v["replica"], v["stream"], v["tick"]) == v["rng"]
        if "value_e3" in v:   # rand.Int() of client entry e=3 at that tick (the value stream)
            assert kat_tick.client_value(v["seed"], v["gid"], v["replica"], v["tick"], 3) == v["value_e3"]


@pytest.mark.parametrize("name", sorted(kat_tick.CASES))
def test_oracle_tick_kat(name):
    kat_tick.run_case(oracle.Oracle, name)
