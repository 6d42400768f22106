#!/usr/bin/env python3
"""Median per-dispatch value of every counter under a rocprofv3 --pmc output tree."""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        tot[c].append(v)
for c, v in sorted(tot.items()):
    print(f"{c:28s} {sorted(v)[len(v) // 2]:.4g}")
