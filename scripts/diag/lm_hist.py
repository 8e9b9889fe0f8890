#!/usr/bin/env python3
"""Line masks of round 2's senders (diagnostic, one MI355X).

Runs rounds 0 and 1 of the bench workload (C4, or C5 with --workload c5) and
reads the Message-Lists: for every vertex the 4-bit mask of its 128-B lines
holding a nonzero word (what round 2's probe reads, up to the few round-0
bits).  Prints the mask histogram weighted by vertices and by out-degree (the
probes: one per arc), and how many bytes a coarser code would gather.

python scripts/diag/lm_hist.py [--workload c5] [--emulate-shard R/N] [rounds (default 2)]
(with a message shard: rows of W = 64 / N words, W / 16 lines each; the
masks of the senders of round `rounds`)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import _gossip_pkg  # noqa: E402


def main():
    argv = sys.argv[1:]
    nr = 2
    if argv and argv[-1].isdigit():
        nr = int(argv.pop())
    args = bench.parse(argv)
    pkg = _gossip_pkg.load()
    n = 1 << args.log2n
    t0 = time.time()
    with pkg.GossipEngine(0, **bench.engine_config(args)) as eng:
        eng.build_chung_lu(n, args.dbar, args.gamma, args.seed)
        origin = pkg.overlay.random_origins(n, args.messages, seed=args.seed)
        er, en = (int(x) for x in args.emulate_shard.split("/")) if args.emulate_shard else (0, 1)
        table = bench.message_table(origin, en, "blocked", lambda o: eng.spread_order(o, hops=3),
                                    pkg.dist.message_shard)
        lo, hi = pkg.dist.message_shard(len(table), en, er)
        eng.set_messages(table[lo:hi])
        eng.reset()
        for _ in range(nr):
            s = eng.round()
            print(f"round {s['round']}: new bits {s['new_bits']}, receivers {s['receivers']}", flush=True)
        deg = eng.degrees().astype(np.float64)
        nib = np.zeros(n, np.uint8)
        chunk = 1 << 21
        seen = eng.seen()   # [n][W] u64
        L = max(1, eng.words // 16)   # 128-B lines per row
        for c in range(0, n, chunk):
            rows = seen[c:c + chunk].reshape(-1, L, eng.words // L)
            nz = (rows != 0).any(axis=2)
            nib[c:c + chunk] = (nz * (1 << np.arange(L))).sum(axis=1).astype(np.uint8)
        del seen
    print(f"read in {time.time() - t0:.1f} s", flush=True)
    lines = np.array([bin(k).count("1") for k in range(16)])
    L = int(nib.max()).bit_length() if nib.any() else 1
    hv = np.bincount(nib, minlength=16)
    ha = np.bincount(nib, weights=deg, minlength=16)
    print("mask  vertices  share   arcs(probes)  share")
    for k in range(16):
        if hv[k]:
            print(f"{k:04b}  {hv[k]:9d}  {hv[k] / n:6.3f}  {ha[k]:13.0f}  {ha[k] / ha.sum():6.3f}")
    act = nib != 0
    exact = (ha * lines).sum()
    top = np.array([0 if k == 0 else int(np.floor(np.log2(k))) + 1 for k in range(16)])   # lines 0..highest
    print(f"active senders {act.sum()} ({act.mean():.3f}), probes on active {ha[1:].sum() / ha.sum():.3f}")
    print(f"lines gathered per probe: exact {exact / ha.sum():.3f}, prefix code (lines 0..highest) "
          f"{(ha * top).sum() / ha.sum():.3f}, whole rows of active senders (<= {L} lines) "
          f"{max(L, 1) * ha[1:].sum() / ha.sum():.3f}")


if __name__ == "__main__":
    main()
