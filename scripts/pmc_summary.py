#!/usr/bin/env python
"""Sum rocprofv3 --pmc counter_collection.csv per (kernel, counter); prints one line per kernel.
Usage: python scripts/pmc_summary.py <file_counter_collection.csv> [kernel-substring]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    n = r["Kernel_Name"]
    if sub not in n:
        continue
    n = re.sub(r"\(anonymous namespace\)::|void ", "", n).split("(")[0][:60]
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[n].add(r["Dispatch_Id"])
for n, cs in agg.items():
    k = len(disp[n])
    print(f"{n}  [{k} dispatches, per dispatch]")
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {v / k:16.0f}")
