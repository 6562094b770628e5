"""raft_stream_probe for the lean kernel's byte mixes at C2 / C2X / C4 sizes
(replicas = ring entries written per element): the device's own rate for the
access shape, against which each line's lean kernel is read.
    python tools/probe_mix.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raft-sample_amd")]
from raftstep.engine import stream_probe  # noqa: E402

out = []
for name, R, n, hb in (("C2 mix, 2^20", 1, 1 << 20, False), ("C2X mix, 2^24", 1, 1 << 24, False),
                       ("C4 mix (R=7 rows), 2^22", 7, 1 << 22, True), ("C4 mix, 2^24", 7, 1 << 24, True)):
    us, by = stream_probe(0, R, n, 20, heartbeat=hb)
    out.append({"mix": name, "replicas": R, "elems": n, "us": us, "bytes": by, "GBs": by / us / 1e3})
    print(json.dumps(out[-1]), flush=True)
