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
    for name, calls, tot, avg, pct in rows_from(path):
        print(f"| `{short(name)}` | {calls} | {tot / 1e6:.3f} | {avg / 1e3:.1f} | {pct:.2f} |")


if __name__ == "__main__":
    main()
