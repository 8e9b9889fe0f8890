"""Early-exit divergence probe (diagnostic): run the wide-rows churn case until
a round diverges; before that round, check the engine's Message-Lists against
the oracle; after it, show a missing receipt and the in-neighbours that carry it."""
import sys
import numpy as np
sys.path.insert(0, ".")
import _gossip_pkg
from oracle import lib as oracle

pkg = _gossip_pkg.load()
rp, col = oracle.chung_lu(60_000, 10, 2.4, 21)
g = pkg.CSR(60_000, rp, col, False)
deg = np.diff(rp)
m = 4096
origin = pkg.overlay.random_origins(g.n, m, seed=21)
inject = (np.arange(m) % 6).astype(np.int32)
ref = oracle.run(g, origin, inject, want_first=True, churn=True, p_fail=0.01, churn_seed=5)
rf = ref["first"]
for rep in range(8):
    eng = pkg.GossipEngine(0, track_first=1, track_digest=1, churn=1, p_fail=0.01, churn_seed=5,
                           hub_threshold=100000, early_exit=1, push_ratio=0.0, sparse_rows=0, unfiltered_pct=0,
                           track_msg_forwards=1)
    eng.load_graph(g)
    eng.set_messages(origin, inject)
    eng.reset()
    for r in range(12):
        first_before = eng.first().copy()
        st = eng.round()
        if st["new_bits"] != ref["stats"][r]["new_bits"]:
            exp_before = rf <= r
            got_before = first_before <= r
            inj = np.zeros_like(exp_before)
            print("rep", rep, "round", r, "diverges", st["new_bits"], ref["stats"][r]["new_bits"], flush=True)
            first = eng.first()
            mism = np.argwhere((first <= r + 1) != (rf <= r + 1))
            mism = np.array([x for x in mism if origin[x[1]] != x[0]])   # receipts, not injections
            print("  expansion mismatches:", len(mism), "eng-has-extra:",
                  int(sum(first[a, b] <= r + 1 for a, b in mism)), flush=True)
            v, k = mism[0]
            nb = col[rp[v]:rp[v + 1]]
            print("  v", v, "msg", k, "deg", deg[v], "eng", first[v, k], "ref", rf[v, k],
                  "seenpop-before", int(got_before[v].sum()), "cmask-size?", flush=True)
            print("  in-neighbours (u, ref first of msg, eng first, deg):",
                  [(int(u), int(rf[u, k]), int(first[u, k]), int(deg[u])) for u in nb], flush=True)
            print("  v's messages held before:", int(got_before[v].sum()), "ref:", int(exp_before[v].sum()),
                  "ref-final:", int((rf[v] < 255).sum()), flush=True)
            break
        if st["new_bits"] == 0 and r >= 5:
            print("rep", rep, "ok", flush=True)
            break
    eng.close()
