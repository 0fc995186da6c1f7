#!/usr/bin/env python3
"""Per-kernel mean of every counter in a tools/pmc_probe.sh output dir.
usage: pmc_table.py DIR [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if keys and not any(k in name for k in keys):
                    continue
                short = name.split("(")[0][:48]
                vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:40s} {sum(v) / len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main()
