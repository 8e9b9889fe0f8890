"""Run the wide-rows parity case in the test-suite order inside one process and
report the first divergence from the oracle in detail (diagnostic)."""
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
modes = [(0.0, 0), (0.0, 1), (1e-12, 90), (10.0, 90)]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ee = int(sys.argv[2]) if len(sys.argv) > 2 else 1
hub = int(sys.argv[3]) if len(sys.argv) > 3 else 512
for rep in range(reps):
    for push, unf in modes:
        for sparse in (0, 1):
            eng = pkg.GossipEngine(0, track_first=1, track_digest=1, churn=1, p_fail=0.01, churn_seed=5,
                                   hub_threshold=hub, early_exit=ee, push_ratio=push, sparse_rows=sparse, unfiltered_pct=unf,
                                   track_msg_forwards=1)
            eng.load_graph(g)
            eng.set_messages(origin, inject)
            eng.reset()
            bad_round = None
            for r in range(60):
                st = eng.round()
                b = ref["stats"][r] if r < len(ref["stats"]) else None
                if b is None or st["new_bits"] != b["new_bits"]:
                    bad_round = (r, st["new_bits"], b and b["new_bits"], st["mode"], st["unfiltered"],
                                 st["sparse_gathered"])
                    break
                if st["new_bits"] == 0 and r >= 5:
                    break
            tag = f"ee={ee} hub={hub} rep{rep} push={push} unf={unf} sparse={sparse}"
            if bad_round is None:
                print(tag, "ok", flush=True)
            else:
                first = eng.first()
                r = bad_round[0]
                ref_first = ref["first"]
                # compare receipts up to round r+1
                mism = np.argwhere((first <= r + 1) != (ref_first <= r + 1))
                vs = np.unique(mism[:, 0])
                print(tag, "DIFF at", bad_round, "vertices", len(vs), "bits", len(mism), flush=True)
                for v in vs[:6]:
                    ks = mism[mism[:, 0] == v][:, 1]
                    print("   v", v, "deg", deg[v], "nbits", len(ks), "eng", first[v, ks[:4]].tolist(),
                          "ref", ref_first[v, ks[:4]].tolist(), flush=True)
            eng.close()
