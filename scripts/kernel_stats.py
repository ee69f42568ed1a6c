#!/usr/bin/env python
"""Per-step kernel time table from a rocprofv3 --kernel-trace --stats CSV directory.

    python scripts/kernel_stats.py gpurun_out/TAG/prof --steps 7 [--title "..."]

--steps = number of training steps inside the profiled run (warmup + timed): every row is
normalised per step.
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_stats.csv under {a.dir}")
    rows = list(csv.DictReader(open(files[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    if a.title:
        print(f"# {a.title}")
    print(f"# {len(rows)} kernels; total GPU kernel time per step: {tot / a.steps / 1e6:.2f} ms")
    print(f"{'ms/step':>9} {'calls/step':>10} {'avg_us':>9} {'%':>6}  kernel")
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[: a.top]:
        t = float(r["TotalDurationNs"])
        n = float(r["Calls"])
        print(f"{t / a.steps / 1e6:9.3f} {n / a.steps:10.1f} {t / n / 1e3:9.1f} {100 * t / tot:6.2f}  {r['Name'][:150]}")


if __name__ == "__main__":
    main()
