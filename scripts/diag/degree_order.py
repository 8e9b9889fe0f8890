"""What an engine-internal degree order of the vertex ids would buy (DESIGN.md
§8 item 2), measured before building it: the C4 overlay as built (randomly
relabelled ids) against the same overlay with ids renumbered by in-degree,
descending (an isomorphic graph loaded through gp_load_graph), same messages
(origins mapped), alternating runs on one GPU.  Per-message outputs are
label-free, so both runs must give the same total sends and round count.

  python3 scripts/diag/degree_order.py [--log2n 24] [--steps 3] [--rounds 2]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def degree_relabel(g):
    """(int2ext, ext2int, row_ptr, col) of g renumbered by in-degree, descending
    (ties by id); each in-list keeps its order, mapped."""
    deg = np.diff(g.row_ptr)
    int2ext = np.argsort(-deg, kind="stable").astype(np.int64)
    ext2int = np.empty_like(int2ext)
    ext2int[int2ext] = np.arange(g.n, dtype=np.int64)
    nd = deg[int2ext]
    rp = np.zeros(g.n + 1, np.int64)
    np.cumsum(nd, out=rp[1:])
    arc = np.repeat(g.row_ptr[:-1][int2ext] - rp[:-1], nd) + np.arange(rp[-1], dtype=np.int64)
    col = ext2int[g.col[arc]].astype(np.int32)
    return int2ext, ext2int, rp, col


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--workload", default="c4")
    a, rest = ap.parse_known_args()
    args = bench.parse(rest + ["--workload", a.workload])
    import _gossip_pkg
    pkg = _gossip_pkg.load()
    n = 1 << args.log2n
    cfg = bench.engine_config(args)
    A = pkg.GossipEngine(0, **cfg)
    A.build_chung_lu(n, args.dbar, args.gamma, args.seed)
    g = A.graph()
    t0 = time.perf_counter()
    int2ext, ext2int, rp, col = degree_relabel(g)
    print(f"relabel {time.perf_counter() - t0:.1f} s", flush=True)
    nnz = g.nnz
    del g
    B = pkg.GossipEngine(0, **cfg)
    B.load_graph(pkg.overlay.CSR(n, rp, col, False))
    del rp, col
    origin = pkg.overlay.random_origins(n, args.messages, seed=args.seed)
    oa = origin[A.spread_order(origin, hops=args.spread_hops)]
    ob = ext2int[origin].astype(np.int32)
    ob = ob[B.spread_order(ob, hops=args.spread_hops)]
    A.set_messages(oa)
    B.set_messages(ob)

    def step(e):
        e.reset()
        st = e.run()
        e.finalize()
        return st

    for name, e in (("random ids", A), ("degree order", B)):
        step(e)
        e.synchronize()
    for r in range(a.rounds):
        for name, e in (("random ids", A), ("degree order", B)):
            e.synchronize()
            t0 = time.perf_counter()
            runs = [step(e) for _ in range(a.steps)]
            e.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            st = runs[-1]
            sends = sum(s["sends"] for s in st)
            per = " ".join(f"r{i}:{'P' if s['mode'] else 'L'}:{s['kernel_ms'] or s['expand_ms']:.2f}"
                           for i, s in enumerate(st))
            print(f"{name:13s} {ms:8.2f} ms  rounds {len(st)} sends {sends} ({sends / nnz:.1f} per arc) | {per}",
                  flush=True)


if __name__ == "__main__":
    main()


if __name__ == "__main__":
    main()
