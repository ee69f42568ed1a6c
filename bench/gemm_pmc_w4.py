#!/usr/bin/env python
"""PMC driver: the W4 kernel (variant 5) vs hipBLASLt on one NT shape (default the M = 65536,
N = 3072, K = 3072 point of bench/gemm_ksweep.py), 3 launches each.  Run under
rocprofv3 --pmc ... --kernel-trace; summarise with scripts/pmc_summary.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext

M, N, K = (int(v) for v in os.environ.get("PMC_SHAPE", "65536,3072,3072").split(","))
a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
ext().gemm_set_variant(5)
for _ in range(3):
    G.gemm_nt(a, b)
ext().gemm_set_variant(0)
for _ in range(3):
    torch.mm(a, b.t())
torch.cuda.synchronize()
