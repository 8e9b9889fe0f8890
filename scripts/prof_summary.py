#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd .db or kernel_stats.csv)
into a small markdown table for profiles/.  usage: prof_summary.py <db|csv> [title]"""
import csv
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"rocprim::ROCPRIM_\d+_NS::", "rocprim::", name)
    if name.startswith("void rocprim") or "rocprim::detail" in name:
        m = re.search(r"detail::(\w+)", name)
        return "rocprim::" + (m.group(1) if m else "kernel")
    return name.split("(")[0].replace("void ", "")


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        # rocpd top_kernels durations are in microseconds -> ns
        return [(r[0], int(r[1]), float(r[2]) * 1e3, float(r[3]) * 1e3, float(r[4]))
                for r in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels")]
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                    float(r["Percentage"])))
    return out


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    print(f"# {title}\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    rows = rows_from(path)
    for name, calls, tot, avg, pct in rows:
        print(f"| `{short(name)}` | {calls} | {tot / 1e6:.3f} | {avg / 1e3:.1f} | {pct:.2f} |")
    # the bench line's roofline kernel set: the pull launch (k_expand /
    # k_expand_flat of width W) plus its hub passes, per pull launch -- what
    # the engine's kernel_ms HIP events bracket
    sets = {}
    for name, calls, tot, avg, pct in rows:
        if short(name).endswith("k_mklm"):   # line masks: W = 64 pull rounds only, inside the pull's events
            sets.setdefault("64", {"launches": 0, "pull_ms": 0.0, "hub_ms": 0.0})["hub_ms"] += tot / 1e6
            continue
        m = re.search(r"k_(expand_flat|expand|hub_partial|hub_final)<(\d+)", short(name))
        if not m:
            continue
        e = sets.setdefault(m.group(2), {"launches": 0, "pull_ms": 0.0, "hub_ms": 0.0})
        if m.group(1).startswith("expand"):
            e["launches"] += calls
            e["pull_ms"] += tot / 1e6
        else:
            e["hub_ms"] += tot / 1e6
    for w, e in sorted(sets.items()):
        if e["launches"]:
            print(f"\nroofline kernel set, W = {w}: k_expand* + (k_mklm +) k_hub_partial + k_hub_final = "
                  f"{e['pull_ms']:.3f} + {e['hub_ms']:.3f} ms over {e['launches']} pull launches = "
                  f"{(e['pull_ms'] + e['hub_ms']) / e['launches']:.3f} ms per launch")


    # per dispatch, from the kernel trace beside the stats: the pull launch as
    # kernel_ms brackets it (a degree-split round's push half before the pull
    # kernel and its k_acc_clear after the hub passes included; push rounds --
    # k_push followed by k_touch_list / k_apply -- excluded)
    import glob
    import os
    trace = glob.glob(os.path.join(os.path.dirname(path), "*kernel_trace.csv"))
    if trace:
        launches, pending, prev = [], 0.0, None
        recs = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
        for r in recs:
            n = short(r["Kernel_Name"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            kd = ("mklm" if "k_mklm" in n else "pull" if "k_expand" in n else "hub" if "k_hub_" in n else
                  "clear" if "k_acc_clear" in n else "push" if ("k_active_list" in n or "k_push" in n) else
                  "apply" if ("k_touch_list" in n or "k_apply" in n) else None)
            if kd is None:
                continue
            if kd == "push":
                pending += dur
            elif kd == "apply":
                pending = 0.0
            elif kd == "mklm" or (kd == "pull" and prev != "mklm"):
                launches.append(dur + pending)
                pending = 0.0
            elif launches:
                launches[-1] += dur
            prev = kd
        if launches:
            print(f"\npull launches from the kernel trace (the kernels kernel_ms brackets, incl. a degree-split "
                  f"round's push half and clear): {len(launches)} launches, {sum(launches):.3f} ms, "
                  f"{sum(launches) / len(launches):.3f} ms per launch")


if __name__ == "__main__":
    main()
