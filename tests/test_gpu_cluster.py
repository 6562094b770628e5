"""GPU: BASELINE config 1 — main.go's 3-node in-process cluster electing a
leader and replicating 10k client entries — through the C++ host layer
(raft-sample_amd/host). The handler-by-handler host loop (shaped like
main.go's goroutines) and the fused raft_tick must end in the same state, and
that state must equal the CPU oracle's after the same number of ticks."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "raft-sample_amd", "lib", "raft_cluster")


def run(mode, entries, seed, period):
    out = subprocess.run([BIN, "--mode", mode, "--entries", str(entries), "--seed", hex(seed),
                          "--client-period", str(period)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr + out.stdout
    return json.loads(out.stdout.strip().splitlines()[-1])


# period 1: SURVEY C1 (one client entry per tick); period 5: main.go:89's one
# write per 10 s at 2 s per tick (main.go:394)
@pytest.mark.parametrize("seed,entries,modes,period", [(0x5EED0001, 10000, ("tick",), 1),
                                                       (0x5EED0001, 10000, ("tick",), 5),
                                                       (0x5EED0001, 600, ("tick", "handlers"), 1),
                                                       (0x5EED0001, 300, ("tick", "handlers"), 5),
                                                       (0x77, 400, ("tick", "handlers"), 1)])
def test_config1_cluster(seed, entries, modes, period):
    import oracle
    res = {m: run(m, entries, seed, period) for m in modes}
    if len(modes) == 2:
        assert res["tick"] == dict(res["handlers"], mode="tick"), res
    r = res["tick"]
    assert r["fault"] == 0 and max(r["commit"]) >= entries and r["leader"].startswith("Server")
    if period > 1:   # a client write every `period` ticks: ~period ticks per committed entry
        assert r["ticks"] >= (entries - 1) * period
    o = oracle.Oracle(replicas=3, groups=1, client_period=period, ring_depth=64, seed=seed)
    o.init_new_nodes(0)
    o.tick(0, r["ticks"])
    s = o.store_state()
    assert list(s["commit"][0]) == r["commit"] and list(s["last"][0]) == r["last"]
    assert int(s["term"][0, 0]) == r["term"]
    assert np.argmax(s["role"][0]) == int(r["leader"][len("Server"):])
