#!/usr/bin/env python
"""Weight-gradient (TN, fp32 accumulate) tile-config A/B on the GPT-2 wgrad shapes at B=64
(K = 65536 tokens): variants 1 (T128), 4 (PP), 5 (W4) and auto.  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench.bench_epilogue import timeit
from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext

K = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
for name, N, D in [("attn_proj", 768, 768), ("qkv", 2304, 768), ("fc", 3072, 768), ("mlp_proj", 768, 3072)]:
    dy, x = r(K, N), r(K, D)
    c = torch.zeros(N, D, device="cuda")
    row = {"shape": name, "M": N, "N": D, "K": K}
    for v, vn in ((0, "auto"), (1, "t128"), (4, "pp"), (5, "w4")):
        ext().gemm_set_variant(v)
        t = timeit(lambda: G.gemm_tn_acc(dy, x, c))
        row[vn] = [round(t * 1e3, 1), round(2.0 * N * D * K / t / 1e9)]
    ext().gemm_set_variant(0)
    print(json.dumps(row), flush=True)
