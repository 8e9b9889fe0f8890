"""C3, per-arc mask engine: after each round r (before round r+1 is run), check
the mask words the round used against a host recomputation from gcol + abits."""
import os, sys, ctypes
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib
pkg = importlib.import_module("gossip-protocol-with-power-law_amd")

n = 1_000_000
eng = pkg.GossipEngine(0, track_digest=1, push_ratio=0.0, unfiltered_pct=0, flat_max_words=0, arc_mask_permille=1)
eng.build_chung_lu(n, 8, 2.5, 3)
origin = pkg.overlay.random_origins(n, 1024, seed=3)
eng.set_messages(origin)
eng.reset()
g = eng.graph()
nnz = g.nnz
nw = (nnz + 63) // 64 + 2
gcol = eng._read(101, np.empty(nnz, np.int32))
for r in range(6):
    st = eng.round()
    am = eng._read(100, np.empty(nw, np.uint64))
    ab = eng._read(102, np.empty((n + 63) // 64, np.uint64))   # abits of round r (k_mkbits of round r)
    act = (ab[gcol >> 6] >> (gcol & 63).astype(np.uint64)) & np.uint64(1)
    pad = np.zeros(((nnz + 63) // 64) * 64, np.uint64)
    pad[:nnz] = act
    bits = pad.reshape(-1, 64) << np.arange(64, dtype=np.uint64)
    ref = np.bitwise_or.reduce(bits, axis=1)
    d = np.nonzero(ref != am[:len(ref)])[0]
    print(r, st["scan"], "words", len(ref), "bad", len(d), flush=True)
    for k in d[:10]:
        hit = np.nonzero(ref == am[k])[0]
        print("   k", k, "k%16", k % 16, "ref", hex(int(ref[k])), "dev", hex(int(am[k])),
              "dev==ref[]", (hit[:5] - k).tolist() if int(am[k]) not in (0, 2**64 - 1) else "-", flush=True)
