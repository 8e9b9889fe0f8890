"""Per-round engine vs oracle counters for one churn configuration (diagnostic).
GOSSIP_HIP_LIB selects the library variant."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import _gossip_pkg  # noqa: E402
from oracle import lib as oracle  # noqa: E402

pkg = _gossip_pkg.load()
m = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rp, col = oracle.chung_lu(60_000, 10, 2.4, 27)
g = pkg.CSR(60_000, rp, col, False)
origin = pkg.overlay.random_origins(g.n, m, seed=27)
cfg = dict(track_first=0, track_digest=1, track_msg_forwards=0, churn=1, p_fail=0.01, churn_seed=8,
           hub_threshold=512, push_ratio=10.0, unfiltered_pct=90, flat_max_words=16, arc_mask_permille=10,
           prefilter_pct=20, compact_rows=0)
eng = pkg.GossipEngine(0, **cfg)
eng.load_graph(g)
eng.set_messages(origin)
eng.reset()
ref = oracle.run(g, origin, churn=True, p_fail=0.01, churn_seed=8, nthreads=8)
for r in range(len(ref["stats"]) + 2):
    st = eng.round()
    b = ref["stats"][r] if r < len(ref["stats"]) else {}
    keys = ("new_bits", "receivers", "sends", "active", "crashed", "removals")
    diff = {k: (st[k], b.get(k)) for k in keys if st[k] != b.get(k)}
    print(r, "mode", st["mode"], "scan", st["scan"], "done_nb", st["done_nb"], "new", st["new_bits"], "DIFF" if diff else "ok", diff,
          flush=True)
    if st["new_bits"] == 0:
        break
