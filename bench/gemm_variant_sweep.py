#!/usr/bin/env python
"""Every gemm.hip tile config (gemm_set_variant) on the GPT-2 B=64 step's epilogue GEMMs
(M = 65536 tokens): fc forward (bias+GELU, pre-activation stored), fc2 / proj forward
(residual + dropout), the fc2 data gradient with the GELU' epilogue.  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench.bench_epilogue import timeit
from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext

M, D = int(os.environ.get("TOKENS", "65536")), 768
r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
C = ext()
names = {1: "T128", 2: "T256", 3: "T2x1", 4: "PP", 5: "W4", 6: "W4_192"}
cases = []
x, w, b = r(M, D), r(4 * D, D), r(4 * D)
aux = torch.empty(M, 4 * D, device="cuda", dtype=torch.bfloat16)
cases.append(("fc_fwd_gelu", 2.0 * M * 4 * D * D, lambda: G.gemm_nt(x, w, bias=b, epi="gelu", pre_out=aux)))
h, w2, b2, res = r(M, 4 * D), r(D, 4 * D), r(D), r(M, D)
cases.append(("fc2_fwd_resid", 2.0 * M * D * 4 * D, lambda: G.gemm_nt(h, w2, bias=b2, epi="resid", resid=res, p=0.1, seed=5)))
wp = r(D, D)
cases.append(("proj_fwd_resid", 2.0 * M * D * D, lambda: G.gemm_nt(x, wp, bias=b2, epi="resid", resid=res, p=0.1, seed=5)))
dy, g = r(M, D), r(M, 4 * D)
w2t = w2.t().contiguous()
cases.append(("fc2_dgrad_gelu_bwd", 2.0 * M * 4 * D * D, lambda: G.gemm_nt(dy, w2t, epi="gelu_bwd", aux=g)))
for name, fl, fn in cases:
    out = {}
    for v in (0, 1, 2, 3, 4, 5, 6):
        C.gemm_set_variant(v)
        try:
            t = timeit(fn)
            out[names.get(v, "auto")] = [round(t * 1e3, 1), round(fl / t / 1e9)]
        except Exception as e:  # a config that does not take this layout
            out[names.get(v, "auto")] = str(e)[:60]
    C.gemm_set_variant(0)
    print(json.dumps({"shape": name, "M": M, "us_tflops": out}), flush=True)
