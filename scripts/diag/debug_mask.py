"""C3 with the per-arc probe vs the per-arc mask, two engines in lockstep:
after every round compare the Message-Lists and print the first vertices that
differ with their in-list geometry."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib
pkg = importlib.import_module("gossip-protocol-with-power-law_amd")

n = 1_000_000
for trial in range(3):
    engs = []
    for am in (0, 1):
        eng = pkg.GossipEngine(0, track_digest=1, push_ratio=0.0, unfiltered_pct=0, flat_max_words=0,
                               arc_mask_permille=am)
        eng.build_chung_lu(n, 8, 2.5, 3)
        origin = pkg.overlay.random_origins(n, 1024, seed=3)
        eng.set_messages(origin)
        eng.reset()
        engs.append(eng)
    g = engs[0].graph()
    rp = g.row_ptr
    bad = False
    for r in range(30):
        s0, s1 = engs[0].round(), engs[1].round()
        a, b = engs[0].seen(), engs[1].seen()
        d = np.nonzero(np.any(a != b, axis=1))[0]
        print(trial, r, s0["new_bits"], s1["new_bits"], s1["scan"], "differ", len(d), flush=True)
        for v in d[:8]:
            print("   v", v, "b", rp[v], "e", rp[v + 1], "deg", rp[v + 1] - rp[v], "b%64", rp[v] % 64,
                  "k0", rp[v] >> 6, "k1", (rp[v + 1] - 1) >> 6,
                  "probe", int(np.unpackbits(a[v].view(np.uint8)).sum()),
                  "mask", int(np.unpackbits(b[v].view(np.uint8)).sum()), flush=True)
        if len(d):
            bad = True
        if s0["new_bits"] == 0:
            break
    for e in engs:
        e.close()
    if bad:
        break
