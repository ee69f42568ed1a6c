#!/usr/bin/env python
"""Weight gradient main_grad += dY^T X (fp32): gemm.hip (split-K, fp32 accumulate) vs the library
GEMM with an fp32 output + add (torch.mm(out_dtype=fp32)), and the bf16-out library GEMM as a
speed bound.  One JSON line per shape."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from bench.bench_wgrad import timeit
from mingpt_distributed_amd.ops import gemm as G


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--D", type=int, default=1600)
    a = ap.parse_args()
    M, D = a.tokens, a.D
    r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
    for name, N, K in [("qkv", 3 * D, D), ("attn_proj", D, D), ("fc", 4 * D, D), ("mlp_proj", D, 4 * D)]:
        dy, x = r(M, N), r(M, K)
        c = torch.zeros(N, K, device="cuda")
        res = {}
        fl = 2.0 * M * N * K
        for tag, fn in [("hip", lambda: G.gemm_tn_acc(dy, x, c)),
                        ("blas_f32_add", lambda: c.add_(torch.mm(dy.t(), x, out_dtype=torch.float32))),
                        ("blas_f32_addmm", lambda: torch.addmm(c, dy.t(), x, out_dtype=torch.float32, out=c)),
                        ("blas_bf16", lambda: torch.mm(dy.t(), x))]:
            try:
                t = timeit(fn)
                res[tag] = [round(t * 1e3, 1), round(fl / t / 1e9)]
            except Exception as e:  # noqa: BLE001
                res[tag] = str(e)[:80]
        print(json.dumps({"wgrad": name, "N": N, "K": K, "M": M, "us_tflops": res}), flush=True)


if __name__ == "__main__":
    main()
