#!/usr/bin/env python
"""Attention kernels alone (GPT-2 shape, B=32) for rocprofv3 --pmc passes: ATTN_ITERS forward
and backward launches at dropout ATTN_P."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mingpt_distributed_amd.ops._ext import ext

B, T, H, hd = int(os.environ.get("ATTN_B", "32")), 1024, 12, 64
p = float(os.environ.get("ATTN_P", "0.1"))
iters = int(os.environ.get("ATTN_ITERS", "2"))
D = H * hd
C = ext()
if hasattr(C, "attention_set_bwd_mode"):  # older builds (A/B) have one schedule
    C.attention_set_bwd_mode(int(os.environ.get("ATTN_BWD_MODE", "0")))
qkv = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
for _ in range(iters):
    out, lse, mask = C.attention_fwd(qkv, B, T, H, p, 1)
    C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, p, 1)
torch.cuda.synchronize()
