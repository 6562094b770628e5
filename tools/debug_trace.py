"""Diagnostic: record a random RAFT-mode event trace on the engine, replay it
on the oracle event by event, and print the first diverging event's request
records and field-level state diff for the diverging groups."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raft-sample_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import harness as H  # noqa: E402
import oracle  # noqa: E402
from raftstep import Engine, abi  # noqa: E402


class Both:
    def __init__(self, **kw):
        self.e, self.o = Engine(**kw), oracle.Oracle(**kw)
        self.cfg = self.e.cfg
        self.n = 0

    def init_new_nodes(self, t):
        self.e.init_new_nodes(t)
        self.o.init_new_nodes(t)

    def _after(self, what, detail):
        de, _ = self.e.state_digest()
        do, _ = self.o.state_digest()
        bad = np.nonzero(de != do)[0]
        self.n += 1
        if bad.size:
            print(f"event {self.n - 1} {what}: groups {bad.tolist()}")
            for g in bad[:3]:
                if detail is not None:
                    print("request(s) for the group:", detail(g))
                print("pre-state engine:")
                for k in abi.STATE_FIELDS:
                    if k.startswith("log"):
                        continue
                    print(" ", k, self.pre_e[k][g].tolist() if self.pre_e[k].ndim > 1 else self.pre_e[k][g])
            se, so = self.e.store_state(), self.o.store_state()
            for g in bad[:3]:
                for k in abi.STATE_FIELDS:
                    if not np.array_equal(se[k][g], so[k][g]):
                        print(f"  g{g} {k}: engine {se[k][g].tolist()} oracle {so[k][g].tolist()}")
            sys.exit(1)

    def _pre(self):
        self.pre_e = self.e.store_state()

    def tick(self, t, k):
        self._pre()
        a, b = self.e.tick(t, k), self.o.tick(t, k)
        assert list(a) == list(b), ("stats", t, k, a, b)
        self._after(f"tick {t}+{k}", None)

    def append_entries(self, now, reqs, ents):
        self._pre()
        a, b = self.e.append_entries(now, reqs, ents), self.o.append_entries(now, reqs, ents)
        assert a.tobytes() == b.tobytes(), "ae resp"
        self._after("ae", lambda g: [r for r in reqs if r["group"] == g])

    def request_vote(self, now, reqs):
        self._pre()
        a, b = self.e.request_vote(now, reqs), self.o.request_vote(now, reqs)
        assert a.tobytes() == b.tobytes(), "vote resp"
        self._after("vote", lambda g: [r for r in reqs if r["group"] == g])

    def group_ops(self, now, ops):
        self._pre()
        a, b = self.e.group_ops(now, ops), self.o.group_ops(now, ops)
        assert a.tobytes() == b.tobytes(), "ops resp"
        self._after(f"ops now={now}", lambda g: [(r, x) for r, x in zip(ops, a) if r["group"] == g])


for sem in (1, 0):
    for seed in range(6):
        rng = np.random.default_rng(40 + sem + 100 * seed)
        b = Both(replicas=5, groups=300, ring_depth=16, client_period=1, seed=0x7ACE + seed, semantics=sem,
                 isolate_per_65536=10000)
        b.init_new_nodes(0)
        H.random_events(b, rng, 60, t0=1)
        print("sem", sem, "seed", seed, "ok", flush=True)
