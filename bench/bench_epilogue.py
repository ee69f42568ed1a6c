#!/usr/bin/env python
"""Epilogue cost microbenchmark: the same GEMM shape with each fused epilogue of the training step
(auto tile config), next to the plain product and hipBLASLt (torch.mm) for the plain product.
Shows what the epilogue VALU / memory work costs on top of the MFMA main loop.  One JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from mingpt_distributed_amd.ops import gemm as G


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
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--D", type=int, default=768)
    a = ap.parse_args()
    M, D = a.tokens, a.D
    r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
    out = {}
    for name, N, K in [("n4d_k1d", 4 * D, D), ("n1d_k4d", D, 4 * D), ("n1d_k1d", D, D), ("n3d_k1d", 3 * D, D)]:
        x, w, b = r(M, K), r(N, K), r(N)
        res = r(M, N)
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        g = r(M, N)
        t = {
            "hipblaslt": timeit(lambda: torch.mm(x, w.t())),
            "none": timeit(lambda: G.gemm_nt(x, w)),
            "bias": timeit(lambda: G.gemm_nt(x, w, bias=b, epi="bias")),
            "gelu": timeit(lambda: G.gemm_nt(x, w, bias=b, epi="gelu", pre_out=aux)),
            "resid_p0": timeit(lambda: G.gemm_nt(x, w, bias=b, epi="resid", resid=res, p=0.0)),
            "resid_p0.1": timeit(lambda: G.gemm_nt(x, w, bias=b, epi="resid", resid=res, p=0.1, seed=5)),
            "gelu_bwd": timeit(lambda: G.gemm_nt(x, w, epi="gelu_bwd", aux=g)),
        }
        if G.frag_aux_ok(M, N, K):  # the fragment-ordered GELU' plane (epilogues 6 / 7)
            fr = torch.empty(G.frag_aux_elems(M, N), device="cuda", dtype=torch.bfloat16)
            G.gemm_nt(x, w, bias=b, epi="gelu", pre_out=fr, frag=True)
            t["gelu_frag"] = timeit(lambda: G.gemm_nt(x, w, bias=b, epi="gelu", pre_out=fr, frag=True))
            # the data gradient through that plane: dz [M, K] = (dy [M, N] x W [N, K]) * GELU'
            dy, wn = r(M, K), r(K, N)
            t["dgrad_none(NN)"] = timeit(lambda: G.gemm_nn(dy, wn))
            t["dgrad_gelu_bwd_frag(NN)"] = timeit(lambda: G.gemm_nn(dy, wn, epi="gelu_bwd", aux=fr, aux_frag=True))
        fl = 2.0 * M * N * K
        out[f"{name}(M={M},N={N},K={K})"] = {k: [round(v * 1e3, 1), round(fl / v / 1e9)] for k, v in t.items()}
    print(json.dumps({"epilogue_us_tflops": out}))


if __name__ == "__main__":
    main()
