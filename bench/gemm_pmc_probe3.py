#!/usr/bin/env python
"""PMC / timing driver for the operand layouts: n^3 GEMM as NT (both k-contiguous) and as the
weight-gradient TN form (both m/n-contiguous, fp32 accumulate) under PP (4) and W4 (5), plus
hipBLASLt.  Prints median ms per case; run under rocprofv3 --pmc ... --kernel-trace for counters."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext
n = int(os.environ.get("PMC_N", "8192"))
iters = int(os.environ.get("PMC_ITERS", "10"))
a = torch.randn(n, n, device="cuda").to(torch.bfloat16)
b = torch.randn(n, n, device="cuda").to(torch.bfloat16)
c = torch.zeros(n, n, device="cuda")


def t(fn):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        s.record(); fn(); e.record()
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in ev)
    return round(2 * n ** 3 / ts[len(ts) // 2] / 1e9, 1)


out = {}
for v, name in ((4, "pp"), (5, "w4")):
    ext().gemm_set_variant(v)
    out["nt_" + name] = t(lambda: G.gemm_nt(a, b))
    out["tn_" + name] = t(lambda: G.gemm_tn_acc(a, b, c))
ext().gemm_set_variant(0)
out["nt_hipblaslt"] = t(lambda: torch.mm(a, b.t()))
out["tn_hipblaslt"] = t(lambda: torch.mm(a.t(), b))
print(json.dumps({f"tflops_n{n}": out}))
