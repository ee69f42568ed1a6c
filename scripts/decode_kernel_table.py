#!/usr/bin/env python
"""Median duration per (kernel, grid) from a rocprofv3 kernel trace (decode profiling)."""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:48]
    d[(n, r["Grid_Size_X"], r["Workgroup_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:14]:
    v.sort()
    print(f"{sum(v)/1000:8.2f} ms  n={len(v):5d}  med {v[len(v)//2]:7.2f} us  min {v[0]:7.2f}  {k[0]} grid={k[1]} wg={k[2]}")
