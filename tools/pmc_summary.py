#!/usr/bin/env python3
"""Per-kernel PMC averages from rocprofv3 *_counter_collection.csv files (one dir per pass)."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        k = re.sub(r"m3::Cfg<(\d+), (\d+), (\d+)> ", r"\1x\2x\3", k).split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:22s} mean {sum(v)/len(v):16.1f}  n={len(v)}")
