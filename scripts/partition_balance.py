"""Per-rank arcs, vertices and ghosts of the C4 overlay (2^24 Chung-Lu, gamma 2.5,
mean degree 16, seed 4, built on the device by gp_build_chung_lu)
under both slice rules of the vertex partition (dist.partition_bounds, mirroring
csrc/xplan.h): equal vertex counts and equal in-arc counts, at
P = 2, 4, 8.  Runs on the GPU box; writes the table to the path given (default
profiles/r03_partition_balance_c4.json)."""
import sys, time, json, numpy as np
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..'))
import _gossip_pkg
pkg = _gossip_pkg.load()
t0 = time.time()
with pkg.GossipEngine(0) as eng:
    eng.build_chung_lu(1 << 24, 16.0, 2.5, 4)
    g = eng.graph()
rp, col = g.row_ptr, g.col
n = 1 << 24
print("built", time.time() - t0, rp[-1], flush=True)
deg = np.diff(rp)
out = {}
for P in (2, 4, 8):
    for rule in ("vertices", "arcs"):
        b = pkg.dist.partition_bounds(n, P, rp if rule == "arcs" else None)
        arcs = [int(rp[e] - rp[s]) for s, e in b]
        verts = [e - s for s, e in b]
        # ghosts per rank: distinct non-owned in-neighbours of owned vertices
        gh = []
        for s, e in b:
            c = col[rp[s]:rp[e]]
            c = c[(c < s) | (c >= e)]
            gh.append(int(np.unique(c).size))
        out[f"{P}-{rule}"] = dict(arcs=arcs, verts=verts, ghosts=gh,
                                  arc_imbalance=max(arcs) / (sum(arcs) / P), vert_imbalance=max(verts) / (n / P))
        print(P, rule, json.dumps(out[f"{P}-{rule}"]), flush=True)
json.dump(out, open('sys.argv[1] if len(sys.argv) > 1 else "profiles/r03_partition_balance_c4.json"', 'w'), indent=1)
