#!/usr/bin/env python3
"""Table of every counter of every pass for the dispatches of one kernel.
usage: pmc_table.py <dir with p0/ p1/ ...> <kernel substring>"""
import csv
import glob
import os
import sys


def main():
    d, kname = sys.argv[1], sys.argv[2]
    cols = {}
    for path in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = {}
        for r in csv.DictReader(open(path)):
            if kname not in r["Kernel_Name"]:
                continue
            per.setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
            per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for c, m in per.items():
            cols[c] = [m[k] for k in sorted(m)]
    names = sorted(cols)
    print("| dispatch | " + " | ".join(names) + " |")
    print("|---" * (len(names) + 1) + "|")
    nd = max(len(v) for v in cols.values()) if cols else 0
    for i in range(nd):
        print(f"| {i} | " + " | ".join(f"{cols[c][i]:.4g}" if i < len(cols[c]) else "" for c in names) + " |")


if __name__ == "__main__":
    main()
