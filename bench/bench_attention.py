#!/usr/bin/env python
"""Attention microbenchmark: gfx950 flash-attention kernels vs torch SDPA (aotriton) on the
GPT-2 shape (B=16, T=1024, H=12, hd=64), causal, with and without dropout.  Random data."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from mingpt_distributed_amd.ops._ext import ext


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--hd", type=int, default=64)
    a = ap.parse_args()
    B, T, H, hd = a.B, a.T, a.H, a.hd
    D = H * hd
    C = ext()
    qkv = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
    dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
    flops_fwd = 4 * B * H * T * T * hd / 2
    for p in (0.0, 0.1):
        out, lse, mask = C.attention_fwd(qkv, B, T, H, p, 1)
        tf = timeit(lambda: C.attention_fwd(qkv, B, T, H, p, 1))
        tb = timeit(lambda: C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, p, 1))
        q, k, v = qkv.view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4).unbind(0)
        q, k, v = (t.contiguous().requires_grad_() for t in (q, k, v))
        go = dout.view(B, T, H, hd).transpose(1, 2).contiguous()
        sf = timeit(lambda: F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=True))
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=True)

        def sdpa_bwd():
            o = F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=True)
            torch.autograd.grad(o, (q, k, v), go)
        sfb = timeit(sdpa_bwd)
        print(json.dumps({"p": p, "mine_fwd_ms": round(tf, 3), "mine_bwd_ms": round(tb, 3),
                          "sdpa_fwd_ms": round(sf, 3), "sdpa_fwd+bwd_ms": round(sfb, 3),
                          "mine_fwd_tflops": round(flops_fwd / tf / 1e9, 1),
                          "mine_bwd_tflops": round(2.5 * flops_fwd / tb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
