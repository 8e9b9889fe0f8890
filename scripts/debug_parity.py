"""Locate the first round/vertex where the engine diverges from the oracle
(diagnostic; usage: python scripts/debug_parity.py [push_ratio] [sparse])."""
import sys
import numpy as np
sys.path.insert(0, ".")
import _gossip_pkg
from oracle import lib as oracle

pkg = _gossip_pkg.load()
push = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
sparse = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ee = int(sys.argv[3]) if len(sys.argv) > 3 else 1
churn = int(sys.argv[4]) if len(sys.argv) > 4 else 1
unf = int(sys.argv[5]) if len(sys.argv) > 5 else 0
rp, col = oracle.chung_lu(60_000, 10, 2.4, 21)
g = pkg.CSR(60_000, rp, col, False)
m = 4096
origin = pkg.overlay.random_origins(g.n, m, seed=21)
inject = (np.arange(m) % 6).astype(np.int32)
kw = dict(churn=True, p_fail=0.01, churn_seed=5) if churn else {}
ref = oracle.run(g, origin, inject, want_first=True, **kw)
eng = pkg.GossipEngine(0, track_first=1, track_digest=1, churn=churn, p_fail=0.01 if churn else 0.0,
                       churn_seed=5, hub_threshold=512, push_ratio=push, sparse_rows=sparse,
                       early_exit=ee, track_msg_forwards=churn, unfiltered_pct=unf)
eng.load_graph(g)
eng.set_messages(origin, inject)
eng.reset()
for r in range(60):
    st = eng.round()
    b = ref["stats"][r] if r < len(ref["stats"]) else None
    diff = {k: (st[k], b[k]) for k in ("new_bits", "sends", "active", "receivers", "crashed", "removals")
            if b is None or st[k] != b[k]}
    print(r, "mode", st["mode"], "sp_g", st["sparse_gathered"], "sp_w", st["sparse_written"],
          "new", st["new_bits"], "DIFF" if diff else "", diff)
    if diff:
        first = eng.first()
        bad = np.argwhere(first != ref["first"])
        print("first-matrix mismatches:", len(bad), bad[:10].tolist())
        for v, k in bad[:5].tolist():
            print(" v", v, "msg", k, "eng", first[v, k], "ref", ref["first"][v, k], "deg", g.row_ptr[v+1]-g.row_ptr[v])
        break
    if st["new_bits"] == 0 and r >= 5:
        break
