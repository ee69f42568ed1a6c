#!/usr/bin/env python
"""Derived per-kernel table from scripts/gpu/step_pmc.sh's two pass summaries (p1.txt, p2.txt):
mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE / 128 (MFMA-busy cycles summed over 1024
SIMDs, GUI_ACTIVE over 8 XCDs), VALU/MFMA and LDS/MFMA instruction ratios, wait/active =
SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY.   python scripts/step_pmc_table.py DIR"""
import re
import sys


def parse(path):
    out, cur = {}, None
    for line in open(path):
        m = re.match(r"^(\S.*?)\s+\[(\d+) dispatches", line)
        if m:
            cur = m.group(1).strip()
            out.setdefault(cur, {"disp": int(m.group(2))})
            continue
        m = re.match(r"^\s+(\w+)\s+([\d.]+)", line)
        if m and cur:
            out[cur][m.group(1)] = float(m.group(2))
    return out


def main():
    d = sys.argv[1]
    a, b = parse(f"{d}/p1.txt"), parse(f"{d}/p2.txt")
    rows = []
    for k in a:
        c = {**a[k], **b.get(k, {})}
        mf = c.get("SQ_INSTS_MFMA", 0.0)
        util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, c.get("GRBM_GUI_ACTIVE", 1.0)) / 128
        rows.append((c.get("SQ_BUSY_CYCLES", 0.0) * c["disp"], k[:60], c["disp"],
                     c.get("SQ_INSTS_VALU", 0.0) / mf if mf else 0.0, util,
                     c.get("SQ_INSTS_LDS", 0.0) / mf if mf else 0.0,
                     c.get("SQ_WAIT_INST_ANY", 0.0) / max(1.0, c.get("SQ_ACTIVE_INST_ANY", 1.0))))
    print(f"{'kernel':60s} {'disp':>5s} {'VALU/MFMA':>9s} {'mfma_util':>9s} {'LDS/MFMA':>8s} {'wait/active':>11s}")
    for _, k, n, vm, u, lm, w in sorted(rows, reverse=True):
        print(f"{k:60s} {n:5d} {vm:9.2f} {100 * u:8.1f}% {lm:8.2f} {w:11.2f}")


if __name__ == "__main__":
    main()
