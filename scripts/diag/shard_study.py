#!/usr/bin/env python3
"""Cost study of message shards at C4 (diagnostic, one MI355X).

1. Builds the C4 overlay once and the bench's spread-ordered message table T
   (4096 messages, bench.message_table with one rank).
2. Arrival matrix: the first-receipt round of every message of T at K vertices
   sampled with probability proportional to their degree (exact: four runs of
   1024 messages with track_first, rows of the sampled vertices kept).
   Saved to OUT/arrival.npz with the per-message features (spread keys, origin
   degree).
3. Times shards of T given as 64-message word ranges [a, a + s) (reset + run +
   finalize, the bench step, median of REPS after one warmup), appending one
   JSON line per shard to OUT/shards.jsonl.

python scripts/diag/shard_study.py [--sizes 6,7,8,9,10] [--samples 8192]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import _gossip_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "shard_study"))
    ap.add_argument("--sizes", default="6,7,8,9,10")
    ap.add_argument("--step", type=int, default=1)
    ap.add_argument("--samples", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-arrival", action="store_true")
    ap.add_argument("--ranges", default="", help="extra a:s word ranges, comma separated")
    ap.add_argument("--sets", default="", help="word sets, ';' separated, each '+'-joined a-b ranges (e.g. 0-6+63)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    pkg = _gossip_pkg.load()
    args = bench.parse([])
    n = 1 << args.log2n
    eng = pkg.GossipEngine(0, **bench.engine_config(args))
    t0 = time.time()
    eng.build_chung_lu(n, args.dbar, args.gamma, args.seed)
    origin = pkg.overlay.random_origins(n, args.messages, seed=args.seed)
    table = bench.message_table(origin, 1, "blocked", lambda o: eng.spread_order(o, hops=3),
                                pkg.dist.message_shard)
    deg = eng.degrees()
    keys = {h: eng.spread_keys(table, hops=h) for h in (1, 2, 3)}
    print(f"overlay + table {time.time() - t0:.1f} s", flush=True)

    if not a.no_arrival:
        rng = np.random.default_rng(7)
        p = deg / deg.sum()
        samp = np.sort(rng.choice(n, size=a.samples, replace=True, p=p)).astype(np.int64)
        arr = np.empty((a.samples, len(table)), np.uint8)
        with pkg.GossipEngine(0, track_first=1, track_digest=0) as fe:
            fe.build_chung_lu(n, args.dbar, args.gamma, args.seed)
            for c in range(0, len(table), 1024):
                fe.set_messages(table[c:c + 1024])
                fe.reset()
                fe.run()
                first = fe.first()
                arr[:, c:c + 1024] = first[samp]
                del first
                print(f"arrival chunk {c} done {time.time() - t0:.1f} s", flush=True)
        np.savez_compressed(os.path.join(a.out, "arrival.npz"), arrival=arr, samples=samp, deg_samples=deg[samp],
                            table=table, origin_deg=deg[table], key1=keys[1], key2=keys[2], key3=keys[3],
                            n=n, nnz=int(deg.sum()))

    ranges = []
    for s in (int(x) for x in a.sizes.split(",") if x):
        ranges += [(w, s) for w in range(0, 64 - s + 1, a.step)]
    for r in (x for x in a.ranges.split(",") if x):
        w, s = (int(y) for y in r.split(":"))
        ranges.append((w, s))
    sets = []
    for spec in (x for x in a.sets.split(";") if x):
        words = []
        for part in spec.split("+"):
            lo, _, hi = part.partition("-")
            words += list(range(int(lo), int(hi or lo) + 1))
        sets.append((spec, words))
    jobs = [(f"{w}:{s}", list(range(w, w + s))) for w, s in ranges] + sets
    f = open(os.path.join(a.out, "shards.jsonl"), "a")
    last = time.time()
    for k, (spec, words) in enumerate(jobs):
        w, s = words[0], len(words)
        eng.set_messages(np.concatenate([table[64 * x:64 * (x + 1)] for x in words]))
        eng.reset()
        eng.run()
        eng.finalize()
        ts, st = [], None
        for _ in range(a.reps):
            eng.synchronize()
            t1 = time.perf_counter()
            eng.reset()
            st = eng.run()
            eng.finalize()
            eng.synchronize()
            ts.append((time.perf_counter() - t1) * 1e3)
        rec = {"spec": spec, "w0": w, "words": s, "W": eng.words, "ms": float(np.median(ts)), "ms_all": ts,
               "rounds": [[x["mode"], round(x["kernel_ms"], 3), round(x["expand_ms"], 3), x["rows_gathered"],
                           x["arcs_scanned"], x["receivers"]] for x in st]}
        f.write(json.dumps(rec) + "\n")
        f.flush()
        if time.time() - last > 30:
            print(f"{k + 1}/{len(jobs)} shards, {time.time() - t0:.1f} s", flush=True)
            last = time.time()
    f.close()
    eng.close()
    print(f"done {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
