#!/usr/bin/env python
"""Tiny driver for PMC collection: runs one NT, one NN and one TN (split-K and not) GEMM of GPT-2
shapes a few times each (use under rocprofv3 --pmc ... --kernel-trace)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mingpt_distributed_amd.ops import gemm as G
M, D = 32768, 768
r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
x, w, dy = r(M, D), r(4 * D, D), r(M, 4 * D)
c = torch.zeros(4 * D, D, device="cuda")
big = r(M, 50304)
cbig = torch.zeros(50304, D, device="cuda")
for _ in range(3):
    G.gemm_nt(x, w)                 # fwd  fc  : 32768 x 3072 x 768
    G.gemm_nn(dy, w)                # dgrad fc : 32768 x 768 x 3072
    G.gemm_tn_acc(dy, x, c)         # wgrad fc : 3072 x 768 x 32768 (split-K)
    G.gemm_tn_acc(big[:, :4096].contiguous(), x, cbig[:4096])  # 4096 x 768 x 32768 (split-K 2)
torch.cuda.synchronize()
