#!/usr/bin/env python3
"""Median per-launch duration of each kernel in a rocprofv3 --kernel-trace CSV (skips the env-reset fills)."""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    print(f"{k:60s} n={len(v):5d} median {statistics.median(v) / 1e3:9.1f} us  mean {statistics.mean(v) / 1e3:9.1f} us")
