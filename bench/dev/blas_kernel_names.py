#!/usr/bin/env python
"""hipBLASLt's kernels for the step's plain GEMM shapes (run under rocprofv3 --kernel-trace --stats:
the kernel names encode the macro tile, MFMA shape and schedule).  NT forward, NN data gradient."""
import torch

r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
M = 131072
for N, K in [(768, 768), (768, 3072), (2304, 768), (3072, 768)]:
    x, w = r(M, K), r(N, K)
    for _ in range(5):
        torch.mm(x, w.t())
    dy, wn = r(M, N), r(N, K)
    for _ in range(5):
        torch.mm(dy, wn)
torch.cuda.synchronize()
