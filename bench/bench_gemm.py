#!/usr/bin/env python
"""GEMM microbenchmark: the hand-written MFMA kernel vs hipBLASLt (torch.mm) on the GPT-2 step
shapes (M = B*T tokens).  Random N(0,1) operands (zero-filled operands inflate MFMA clocks).
Prints one JSON line per shape."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from mingpt_distributed_amd.ops import gemm as G


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
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--V", type=int, default=50257)
    a = ap.parse_args()
    M, D, V = a.tokens, a.D, a.V
    Vp = (V + 127) // 128 * 128
    r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
    rows = []
    C = __import__("mingpt_distributed_amd.ops._ext", fromlist=["ext"]).ext()

    def both(fn):  # A/B the tile configs of the hand-written kernel in one process
        out = []
        for v in VARIANTS.values():
            C.gemm_set_variant(v)
            out.append(timeit(fn))
        C.gemm_set_variant(0)
        return out[0], out

    variants = {}
    for name, N, K in [("qkv", 3 * D, D), ("attn_proj", D, D), ("fc", 4 * D, D), ("mlp_proj", D, 4 * D),
                       ("lm_head", V, D)]:
        x, w = r(M, K), r(N, K)
        ld = Vp if name == "lm_head" else None
        t_mine, variants[("fwd", name)] = both(lambda: G.gemm_nt(x, w, ld=ld))
        t_blas = timeit(lambda: torch.mm(x, w.t()))
        rows.append(("fwd_nt", name, M, N, K, t_mine, t_blas))
        # dgrad: dx[M,K] = dy[M,N] @ w[N,K]
        dy = r(M, Vp if name == "lm_head" else N)
        if name == "lm_head":
            dy[:, V:] = 0
        t_mine, variants[("dgrad", name)] = both(lambda: G.gemm_nn(dy, w))
        dyv = dy[:, :N] if name == "lm_head" else dy
        t_blas = timeit(lambda: torch.mm(dyv, w))
        rows.append(("dgrad_nn", name, M, K, N, t_mine, t_blas))
        # wgrad: dw[N,K] += dy^T x
        c = torch.zeros(N, K, device="cuda")
        t_mine, variants[("wgrad", name)] = both(lambda: G.gemm_tn_acc(dy, x, c, n_valid=N))
        t_blas = timeit(lambda: torch.mm(dyv.t(), x))
        rows.append(("wgrad_tn", name, N, K, M, t_mine, t_blas))
    tot_m = tot_b = 0.0
    for kind, name, m, n, k, tm, tb in rows:
        fl = 2.0 * m * n * k
        tot_m += tm
        tot_b += tb
        print(json.dumps({"kind": kind, "layer": name, "M": m, "N": n, "K": k, "mine_ms": round(tm, 4),
                          "hipblaslt_ms": round(tb, 4), "mine_tflops": round(fl / tm / 1e9, 1),
                          "hipblaslt_tflops": round(fl / tb / 1e9, 1), "speedup": round(tb / tm, 3)}),
              flush=True)
    print(json.dumps({"total_mine_ms": round(tot_m, 3), "total_hipblaslt_ms": round(tot_b, 3)}))
    print(json.dumps({"variant_ms(" + ",".join(VARIANTS) + ")": {f"{k[0]}:{k[1]}": [round(t, 4) for t in v] for k, v in variants.items()}}))
    # fused-epilogue shapes of the step (forward and NT data-gradient forms), all tile configs
    epi = {}
    bias3, bias4 = r(3 * D), r(4 * D)
    x, wq, wfc, wp = r(M, D), r(3 * D, D), r(4 * D, D), r(D, 4 * D)
    u, pre = r(M, 4 * D), torch.empty(M, 4 * D, device="cuda", dtype=torch.bfloat16)
    dz, wpt = r(M, D), G.transpose(wp, D)
    _, epi["qkv_bias"] = both(lambda: G.gemm_nt(x, wq, bias=bias3, epi="bias"))
    _, epi["fc_gelu"] = both(lambda: G.gemm_nt(x, wfc, bias=bias4, epi="gelu", pre_out=pre))
    _, epi["proj_resid_drop"] = both(lambda: G.gemm_nt(u, wp, bias=r(D), epi="resid", resid=x, p=0.1, seed=3))
    _, epi["dgrad_gelu_bwd_nt"] = both(lambda: G.gemm_nt(dz, wpt, epi="gelu_bwd", aux=pre))
    _, epi["dgrad_fc_nt"] = both(lambda: G.gemm_dgrad(u, wfc, wt=G.transpose(wfc, 4 * D)))
    print(json.dumps({"epilogue_ms(" + ",".join(VARIANTS) + ")": {k: [round(t, 4) for t in v] for k, v in epi.items()}}))
    for n in (4096, 8192):
        a4, b4 = r(n, n), r(n, n)
        t4, v4 = both(lambda: G.gemm_nt(a4, b4))
        tb4 = timeit(lambda: torch.mm(a4, b4.t()))
        print(json.dumps({f"gemm_{n}^3_tflops": {k: round(2 * n ** 3 / t / 1e9, 1) for k, t in zip(VARIANTS, v4)} |
                          {"hipblaslt": round(2 * n ** 3 / tb4 / 1e9, 1)}}))


if __name__ == "__main__":
    main()
