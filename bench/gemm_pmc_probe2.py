#!/usr/bin/env python
"""PMC driver: 8192^3 NT GEMM under each tile config (T256 = variant 2, ping-pong = 4) and
hipBLASLt (torch.mm), 3 launches each.  Run under rocprofv3 --pmc ... --kernel-trace."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext
n = int(os.environ.get("PMC_N", "8192"))
a = torch.randn(n, n, device="cuda").to(torch.bfloat16)
b = torch.randn(n, n, device="cuda").to(torch.bfloat16)
for v in (2, 4):
    ext().gemm_set_variant(v)
    for _ in range(3):
        G.gemm_nt(a, b)
ext().gemm_set_variant(0)
for _ in range(3):
    torch.mm(a, b.t())
torch.cuda.synchronize()
