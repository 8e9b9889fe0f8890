"""Repeat one parity configuration N times in one process and report any
divergence from the oracle (diagnostic for nondeterministic mismatches)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import _gossip_pkg
from oracle import lib as oracle

pkg = _gossip_pkg.load()
push = float(sys.argv[1]); sparse = int(sys.argv[2]); reps = int(sys.argv[3])
ee = int(sys.argv[4]) if len(sys.argv) > 4 else 1
hub = int(sys.argv[5]) if len(sys.argv) > 5 else 512
rp, col = oracle.chung_lu(60_000, 10, 2.4, 21)
g = pkg.CSR(60_000, rp, col, False)
m = 4096
origin = pkg.overlay.random_origins(g.n, m, seed=21)
inject = (np.arange(m) % 6).astype(np.int32)
kw = dict(churn=True, p_fail=0.01, churn_seed=5)
ref = oracle.run(g, origin, inject, want_first=True, **kw)
eng = pkg.GossipEngine(0, track_first=1, track_digest=1, churn=1, p_fail=0.01, churn_seed=5,
                       hub_threshold=hub, push_ratio=push, sparse_rows=sparse, track_msg_forwards=1,
                       early_exit=ee)
eng.load_graph(g)
eng.set_messages(origin, inject)
for rep in range(reps):
    eng.reset()
    bad = None
    for r in range(40):
        st = eng.round()
        b = ref["stats"][r] if r < len(ref["stats"]) else None
        if b is None or any(st[k] != b[k] for k in ("new_bits", "sends", "active", "receivers")):
            bad = (r, st["new_bits"], b and b["new_bits"], st["mode"], st["sparse_gathered"], st["sparse_written"])
            first = eng.first()
            mism = np.argwhere(first != ref["first"])
            print("rep", rep, "DIVERGE at round", bad, "first mismatches", len(mism), mism[:8].tolist(),
                  [(int(first[v, k]), int(ref["first"][v, k])) for v, k in mism[:8].tolist()], flush=True)
            break
        if st["new_bits"] == 0 and r >= 5:
            break
    if bad is None:
        ok = np.array_equal(eng.first(), ref["first"]) and np.array_equal(eng.digest(), ref["digest"])
        print("rep", rep, "ok" if ok else "FIRST/DIGEST MISMATCH", "rounds", r + 1, "ref", ref["rounds"], flush=True)
