"""Diagnostic: the (200 messages, explicit crashes, track_msg_forwards) case of
test_finalize_paths_agree, per round against the oracle, under the library
GOSSIP_HIP_LIB and a few configurations."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import _gossip_pkg  # noqa: E402
from oracle import lib as oracle  # noqa: E402

pkg = _gossip_pkg.load()
g = pkg.overlay.barabasi_albert(3000, 2, seed=11)
m = int(sys.argv[1]) if len(sys.argv) > 1 else 200
origin = pkg.overlay.random_origins(g.n, m, seed=11)
crashes = [(int(v), 2) for v in range(100, 3000, 300)]
ref = oracle.run(g, origin, crashes=crashes)
for tag, extra in (("default", {}), ("split0", dict(split_deg=0)), ("pull", dict(push_ratio=0.0)),
                   ("ee0", dict(early_exit=0))):
    cfg = dict(track_digest=1, track_msg_forwards=1, **extra)
    with pkg.GossipEngine(0, **cfg) as eng:
        eng.load_graph(g)
        eng.set_messages(origin)
        eng.reset()
        stats = []
        for r in range(254):
            if r == 2:
                eng.crash([v for v, _ in crashes])
            st = eng.round()
            stats.append(st)
            if st["new_bits"] == 0:
                break
        eng.finalize()
        fwd = eng.forwards()
        cov = eng.coverage()
    bad = [(a["round"], k, a[k], b[k]) for a, b in zip(stats, ref["stats"])
           for k in ("new_bits", "receivers", "sends", "active", "crashed", "removals") if a[k] != b[k]]
    print(tag, "rounds", len(stats), ref["rounds"], "cov ok", np.array_equal(cov, ref["coverage"]),
          "fwd ok", np.array_equal(fwd, ref["forwards"]), "fwd diff", int((fwd.astype(np.int64) - ref["forwards"].astype(np.int64)).sum()),
          "modes", "".join("P" if s["mode"] else ("L%d" % s["scan"]) for s in stats), "bad", bad[:6], flush=True)
