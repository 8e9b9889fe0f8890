"""After round 1 of C4: how many nonzero words do the senders of round 2 hold,
weighted by how often round 2 gathers them (out-degree)?"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib
pkg = importlib.import_module("gossip-protocol-with-power-law_amd")
n = 1 << 24
eng = pkg.GossipEngine(0, track_digest=0, track_first=0)
eng.build_chung_lu(n, 16.0, 2.5, 4)
origin = pkg.overlay.random_origins(n, 4096, seed=4)
eng.set_messages(origin)
eng.reset()
for r in range(2):
    st = eng.round()
    print(r, st["new_bits"], st["receivers"], flush=True)
fpop = eng._read(11, np.empty(n, np.uint32))      # senders of round 2
g = eng.graph()
outdeg = np.diff(g.row_ptr)                        # undirected: in == out
act = np.nonzero(fpop)[0]
seen = np.empty((n, 64), np.uint64)
eng._read(0, seen)
nzw = np.count_nonzero(seen[act], axis=1)
bits = np.unpackbits(seen[act].view(np.uint8), axis=1).sum(axis=1)
w = outdeg[act].astype(np.float64)
for cap in (7, 15, 23, 31):
    print("cap", cap, "senders", round(float((nzw <= cap).mean()), 3), "gathers", round(float(w[nzw <= cap].sum() / w.sum()), 3), flush=True)
print("mean bits", bits.mean(), "weighted", (bits * w).sum() / w.sum())
