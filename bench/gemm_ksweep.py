#!/usr/bin/env python
"""Per-tile fixed cost of the forward GEMM: time(K) at fixed M, N for K = 768 .. 6144.  The slope
is the main-loop cost per K, the intercept the prologue + epilogue cost the K loop does not hide.
One JSON line per (N, epilogue)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from mingpt_distributed_amd.ops import gemm as G
from bench.bench_epilogue import timeit


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
    for N in (3072, 768):
        for epi in ("none", "bias", "gelu"):
            row = {"M": M, "N": N, "epi": epi}
            for K in (768, 1536, 3072, 6144):
                x, w, b = r(M, K), r(N, K), r(N)
                aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                if epi == "none":
                    f = lambda: G.gemm_nt(x, w)
                elif epi == "bias":
                    f = lambda: G.gemm_nt(x, w, bias=b, epi="bias")
                else:
                    f = lambda: G.gemm_nt(x, w, bias=b, epi="gelu", pre_out=aux)
                t = timeit(f)
                row[f"K{K}"] = [round(t * 1e3, 1), round(2.0 * M * N * K / t / 1e9)]
                if epi == "none":
                    row[f"blas_K{K}"] = round(timeit(lambda: torch.mm(x, w.t())) * 1e3, 1)
                del x, w, aux
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
