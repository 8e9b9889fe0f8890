#!/usr/bin/env python3
"""Per-launch HBM traffic of the pull (k_expand / k_expand_flat and the hub
passes k_hub_partial / k_hub_final that follow it: the kernel set the bench
line's roofline and the engine's kernel_ms cover) from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in KB; they cannot share a pass on gfx950) next to
the algorithmic bytes of the same rounds (bench.round_bytes).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts the
128-B read requests at 64 B, so fetched bytes = 2 x FETCH_SIZE x 1024
(checked here: TCC_EA0_RDREQ_128B x 128 B gives the same figure).  Infinity
Cache hits are counted, not excluded, so this is L2-to-fabric traffic.

usage: pmc_summary.py <dir holding fetch/ write/ and fetch.err> [json_out]"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


SET = ("k_mklm", "k_expand", "k_hub_partial", "k_hub_final", "k_acc_clear",
       "k_active_list", "k_push", "k_touch_list", "k_apply")


def _kind(name):
    for key, kind in (("k_mklm", "mklm"), ("k_expand", "pull"), ("k_hub_", "hub"), ("k_acc_clear", "clear"),
                      ("k_active_list", "push"), ("k_push", "push"), ("k_touch_list", "apply"), ("k_apply", "apply")):
        if key in name:
            return kind
    return None


def load(d, counter):
    """Counter per pull launch -- the kernels kernel_ms brackets: a k_expand*
    dispatch opens a launch unless the line-mask pass k_mklm just opened it (it
    runs first, inside the pull's events); the hub dispatches and a
    degree-split round's k_acc_clear after it add to it, and so does the push
    half before it (k_active_list / k_push / k_push_big directly followed by
    the pull; push rounds are followed by k_touch_list / k_apply instead and
    are not counted)."""
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per, kind = {}, {}
    for r in csv.DictReader(open(path)):
        kd = _kind(r["Kernel_Name"])
        if r["Counter_Name"] != counter or kd is None:
            continue
        k = int(r["Dispatch_Id"])
        per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
        kind[k] = kd
    out = []
    prev, pending = None, 0.0
    for k in sorted(per):
        kd = kind[k]
        if kd == "push":
            pending += per[k]
        elif kd == "apply":
            pending = 0.0
        elif kd == "mklm" or (kd == "pull" and prev != "mklm"):
            out.append(per[k] + pending)
            pending = 0.0
        elif out:
            out[-1] += per[k]
        prev = kd
    return out


def main():
    d = sys.argv[1]
    fetch = load(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = load(os.path.join(d, "write"), "WRITE_SIZE")
    rounds = [json.loads(l) for l in open(os.path.join(d, "fetch.err")) if l.startswith("{")]
    bench = json.loads(open(os.path.join(d, "fetch.json")).read())
    from bench import round_bytes
    words = bench["config"]["words_per_row"]
    n = bench["config"]["n"]
    pull = [r for r in rounds if r["mode"] == 0 and r.get("kernel_ms", 0) > 0]
    assert len(pull) == len(fetch) == len(write), (len(pull), len(fetch), len(write))
    rows = []
    for r, f, w in zip(pull, fetch, write):
        rows.append({"round": r["round"], "alg_GB": round_bytes(r, words, n) / 1e9,
                     "fetch_GB": 2 * f * 1024 / 1e9, "write_GB": w * 1024 / 1e9,
                     "kernel_ms": r["kernel_ms"]})
    print("| round | alg GB | fetch GB (2 x FETCH_SIZE) | write GB | HBM GB | HBM / alg | kernel ms | HBM TB/s |")
    print("|---|---|---|---|---|---|---|---|")
    for x in rows:
        h = x["fetch_GB"] + x["write_GB"]
        print(f"| {x['round']} | {x['alg_GB']:.2f} | {x['fetch_GB']:.2f} | {x['write_GB']:.2f} | {h:.2f} | "
              f"{h / x['alg_GB']:.3f} | {x['kernel_ms']:.2f} | {h / x['kernel_ms']:.2f} |")
    ta = sum(x["alg_GB"] for x in rows)
    th = sum(x["fetch_GB"] + x["write_GB"] for x in rows)
    tm = sum(x["kernel_ms"] for x in rows)
    print(f"| all {len(rows)} launches | {ta:.2f} | | | {th:.2f} | {th / ta:.3f} | {tm:.2f} | {th / tm:.2f} |")
    out = {"kernel": "k_mklm (line-mask rounds) + k_expand + k_hub_partial + k_hub_final (+ a degree-split round's "
                     "push half and k_acc_clear)", "launches": len(rows), "traffic_bytes_per_launch": th * 1e9 / len(rows),
           "alg_bytes_per_launch": ta * 1e9 / len(rows), "kernel_ms_per_launch": tm / len(rows),
           "rounds": rows, "config": bench["config"],
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bytes = "
                     "2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md gfx950 correction)"}
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
