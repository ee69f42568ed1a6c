#!/usr/bin/env python
"""Weight-gradient GEMM microbenchmark (fp32 accumulate, split-K): every tile config on the
GPT-2 wgrad shapes at M = tokens.  One JSON line per shape: ms and TFLOP/s per variant."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext

VARIANTS = {"auto": 0, "t128": 1, "w4": 5, "w4n192": 6}  # gemm_set_variant codes


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in ev)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--variants", default="0,1,5")
    a = ap.parse_args()
    M, D = a.tokens, a.D
    r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
    C = ext()
    for name, N, K in [("qkv", 3 * D, D), ("attn_proj", D, D), ("fc", 4 * D, D), ("mlp_proj", D, 4 * D),
                       ("lm_head", 50304, D)]:
        dy, x = r(M, N), r(M, K)
        c = torch.zeros(N, K, device="cuda")
        res = {}
        for v in map(int, a.variants.split(",")):
            C.gemm_set_variant(v)
            t = timeit(lambda: G.gemm_tn_acc(dy, x, c))
            res[{c: n for n, c in VARIANTS.items()}[v]] = [round(t * 1e3, 1), round(2.0 * M * N * K / t / 1e9)]
        C.gemm_set_variant(0)
        res["hipblaslt"] = [round(timeit(lambda: torch.mm(dy.t(), x)) * 1e3, 1)]
        print(json.dumps({"wgrad": name, "N": N, "K": K, "M": M, "us_tflops": res}), flush=True)


if __name__ == "__main__":
    main()
