#!/usr/bin/env python
"""Per-(kernel, grid) breakdown of ONE training step from a rocprofv3 kernel trace.

The last full step is the span between the last two optimizer (adamw) launches.
Usage: python scripts/step_breakdown.py <prof_dir>/run_kernel_trace.csv [top]
"""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([\w:]+(<[^()]*>)?)", name)
    return (m.group(1) if m else name)[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    idx = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    a, b = idx[-2] + 1, idx[-1] + 1
    agg = collections.OrderedDict()
    tot = 0.0
    for r in rows[a:b]:
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]),
               int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        e = agg.setdefault(key, [0, 0.0])
        e[0] += 1
        e[1] += d
    span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    print(f"# one step: kernel time {tot / 1e3:.2f} ms, span {span / 1e3:.2f} ms")
    print("#   total_us calls  avg_us  blocks_x,y,z  kernel")
    for k, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{d:10.1f} {c:5d} {d / c:7.1f}  {k[1]},{k[2]},{k[3]}  {k[0]}")


if __name__ == "__main__":
    main()
