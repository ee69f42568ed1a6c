#!/usr/bin/env python
"""Attention fwd/bwd timing at the bench shape for one-box A/B of extension builds
(MINGPT_EXT_SO=build/ab/<name>/_C.so); prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mingpt_distributed_amd.ops._ext import ext

B, T, H, hd = int(os.environ.get("ATTN_B", "64")), 1024, 12, 64
C = ext()
D = H * hd
qkv = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


out, lse, mask = C.attention_fwd(qkv, B, T, H, 0.1, 1)
print(json.dumps({"so": os.environ.get("MINGPT_EXT_SO", "tree"), "B": B,
                  "fwd_ms": round(timeit(lambda: C.attention_fwd(qkv, B, T, H, 0.1, 1)), 4),
                  "bwd_ms": round(timeit(lambda: C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, 0.1, 1)), 4)}))
