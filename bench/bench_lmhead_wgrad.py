#!/usr/bin/env python
"""LM-head weight gradient at the B=64 step shape: gemm.hip TN (fp32 accumulate into main_grad,
split-K) vs hipBLASLt (torch.mm with an fp32 output, then added into main_grad)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mingpt_distributed_amd.ops import gemm as G


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


M, V, Vp, D = 65536, 50257, 50304, 768
dl = (torch.randn(M, Vp, device="cuda") * 0.01).to(torch.bfloat16)
dl[:, V:] = 0
h = torch.randn(M, D, device="cuda").to(torch.bfloat16)
mg = torch.zeros(V, D, device="cuda")
ours = t(lambda: G.gemm_tn_acc(dl, h, mg, n_valid=V))
blas = t(lambda: mg.add_(torch.mm(dl[:, :V].t(), h, out_dtype=torch.float32)))
blas2 = t(lambda: torch.addmm(mg, dl[:, :V].t(), h, out_dtype=torch.float32, out=mg) if False else
          mg.add_(torch.mm(dl.t(), h, out_dtype=torch.float32)[:V]))
print(json.dumps({"lm_head_wgrad_ms": {"gemm_hip_tn_acc": round(ours, 3), "hipblaslt_mm_f32_add": round(blas, 3),
                                       "hipblaslt_padded": round(blas2, 3)}}))
