#!/usr/bin/env python
"""Per-kernel register / spill summary and instruction counts from a hipcc --save-temps .s file.

    python scripts/isa_stats.py gemm-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter] [--count a,b,c]
"""
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--count")]
cnt = [a.split("=", 1)[1].split(",") for a in sys.argv[1:] if a.startswith("--count=")]
cnt = cnt[0] if cnt else ["s_and_saveexec", "v_readfirstlane", "v_mfma", "buffer_load", "ds_read", "s_barrier",
                          "scratch_"]
s = open(args[0]).read()
filt = args[1] if len(args) > 1 else ""
bodies = {}
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    end = s.find(".Lfunc_end", m.end())
    bodies[m.group(1)] = s[m.end():end]
meta = s[s.find("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or filt not in name.group(1):
        continue
    g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]
    body = bodies.get(name.group(1), "")
    counts = " ".join(f"{c}={body.count(c)}" for c in cnt)
    print(f"{name.group(1)[18:88]:70s} vgpr={g('vgpr_count')} agpr={g('agpr_count')} "
          f"spill={g('vgpr_spill_count')} | {counts}")
