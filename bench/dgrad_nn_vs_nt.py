#!/usr/bin/env python
"""Data gradients dX = dY @ W at the GPT-2 B=64 shapes: NN layout straight from the stored weight
(gemm.hip layout 1; tile config auto / forced W4 / PP) vs NT against a per-step transposed copy
(ops/gemm.gemm_dgrad, transpose included).  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench.bench_epilogue import timeit
from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext

M, D = 65536, 768
r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
C = ext()
for nm, n_in, n_out in (("proj", D, D), ("fc", D, 4 * D), ("qkv", D, 3 * D), ("fc2_gelu", 4 * D, D)):
    dy, w = r(M, n_out), r(n_out, n_in)
    aux = r(M, n_in) if nm == "fc2_gelu" else None
    epi = "gelu_bwd" if aux is not None else "none"
    out = {"nt_transpose": round(timeit(lambda: G.gemm_dgrad(dy, w, epi=epi, aux=aux)) * 1e3, 1)}
    for v, name in ((0, "nn_auto"), (1, "nn_T128"), (5, "nn_W4")):
        C.gemm_set_variant(v)
        out[name] = round(timeit(lambda: G.gemm_nn(dy, w, epi=epi, aux=aux)) * 1e3, 1)
    C.gemm_set_variant(0)
    ref = (dy.float() @ w.float())
    err = (G.gemm_nn(dy, w).float() - ref).abs().max().item() / ref.abs().max().item() if aux is None else 0.0
    print(json.dumps({"shape": nm, "M": M, "N": n_in, "K": n_out, "us": out, "nn_rel_err": round(err, 4)}), flush=True)
