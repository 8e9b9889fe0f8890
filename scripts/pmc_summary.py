#!/usr/bin/env python3
"""Per-dispatch HBM traffic of the gossip kernels from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; KB units) next to the algorithmic bytes of each round.
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the
bytes of wide coalesced reads, so fetched bytes = 2 x FETCH_SIZE x 1024.
usage: pmc_summary.py <dir with fetch/ write/ subdirs and fetch.err>"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def load(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.append((int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
                    float(r["Counter_Value"])))
    out.sort()
    return out


def main():
    d = sys.argv[1]
    fetch = load(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = load(os.path.join(d, "write"), "WRITE_SIZE")
    rounds = [json.loads(l) for l in open(os.path.join(d, "fetch.err")) if l.startswith("{")]
    from bench import round_bytes
    words = 64
    n = 1 << 24
    ex_f = [(k, v) for _, k, v in fetch if "k_expand" in k]
    ex_w = [(k, v) for _, k, v in write if "k_expand" in k]
    pull = [r for r in rounds if r["mode"] == 0]
    print("| round | kernel | alg GB | fetch GB (2x FETCH_SIZE) | write GB | HBM GB | HBM / alg |")
    print("|---|---|---|---|---|---|---|")
    tot_a = tot_h = 0.0
    for r, (k, f), (_, w) in zip(pull, ex_f, ex_w):
        alg = round_bytes(r, words, n) / 1e9
        fg, wg = 2 * f * 1024 / 1e9, w * 1024 / 1e9
        tot_a += alg
        tot_h += fg + wg
        print(f"| {r['round']} | {k} | {alg:.2f} | {fg:.2f} | {wg:.2f} | {fg + wg:.2f} | {(fg + wg) / alg:.3f} |")
    print(f"| all pull | k_expand | {tot_a:.2f} | | | {tot_h:.2f} | {tot_h / max(tot_a, 1e-9):.3f} |")
    print()
    agg = {}
    for lst, key in ((fetch, "f"), (write, "w")):
        for _, k, v in lst:
            a = agg.setdefault(k, {"f": 0.0, "w": 0.0, "n": 0})
            a[key] += v
            if key == "f":
                a["n"] += 1
    print("| kernel | dispatches | fetch GB (2x) | write GB |")
    print("|---|---|---|---|")
    for k, a in sorted(agg.items(), key=lambda x: -x[1]["f"]):
        print(f"| `{k}` | {a['n']} | {2 * a['f'] * 1024 / 1e9:.2f} | {a['w'] * 1024 / 1e9:.2f} |")


if __name__ == "__main__":
    main()
