"""Per-round counters of a churn run over a P-way vertex partition (group
mode: device copies, gp_round_group) against the oracle (diagnostic for the
W = 64 churn case of tests/rccl_standin_driver.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import _gossip_pkg  # noqa: E402
from oracle import lib as oracle  # noqa: E402

pkg = _gossip_pkg.load()
P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
by_arcs = int(sys.argv[2]) if len(sys.argv) > 2 else 0
extra = dict(a.split("=") for a in sys.argv[3:])
rp, col = oracle.chung_lu(50_000, 10, 2.4, 19)
g = pkg.CSR(50_000, rp, col, False)
origin = pkg.overlay.random_origins(g.n, 4096, seed=19)
inject = (np.arange(4096) % 3).astype(np.int32)
ref = oracle.run(g, origin, inject, churn=True, p_fail=0.01, churn_seed=6, nthreads=8)
cfg = dict(track_first=0, track_msg_forwards=1, churn=1, p_fail=0.01, churn_seed=6, hub_threshold=512,
           partition_by_arcs=by_arcs)
cfg.update({k: int(v) for k, v in extra.items()})
engs = []
for k in range(P):
    e = pkg.GossipEngine(0, **cfg)
    e.load_graph(g)
    e.set_partition(k, P)
    e.set_messages(origin, inject)
    e.reset()
    engs.append(e)
keys = ("new_bits", "receivers", "sends", "active", "crashed", "removals", "reports")
for r in range(len(ref["stats"]) + 2):
    st = pkg.GossipEngine.round_group(engs)
    b = ref["stats"][r] if r < len(ref["stats"]) else {}
    diff = {k: (st[k], b.get(k)) for k in keys if st[k] != b.get(k)}
    print(r, "mode", st["mode"], "scan", st["scan"], "new", st["new_bits"], "DIFF" if diff else "ok", diff, flush=True)
    if st["new_bits"] == 0 and r >= 2:
        break
