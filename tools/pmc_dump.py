#!/usr/bin/env python3
"""Mean of every PMC counter per kernel (substring filter) from a rocprofv3 counter_collection.csv tree
(tuning tool).   python tools/pmc_dump.py DIR [--kernel mmql]"""
import argparse
import collections
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--kernel", default="")
a = ap.parse_args()
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if a.kernel in k:
            acc[(k[:90], row["Counter_Name"])].append(float(row["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k}  {c:28s} n={len(v):4d} mean={sum(v) / len(v):.1f}")
