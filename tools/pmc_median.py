#!/usr/bin/env python3
"""Median per-dispatch PMC values per kernel (millions) for each variant dir under a PMC output root."""
import collections
import csv
import glob
import os
import re
import statistics
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*/"))):
    rows = []
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = re.sub(r".*::(k_\w+)<.*", r"\1", r["Kernel_Name"])
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")))
    for k, v in sorted(agg.items()):
        if k.startswith("k_"):
            print(f"   {k:18s}", " ".join(f"{c.replace('SQ_', '')}={statistics.median(x) / 1e6:.2f}M" for c, x in sorted(v.items())))
