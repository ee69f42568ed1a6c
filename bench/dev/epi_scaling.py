#!/usr/bin/env python
"""Is the residual epilogue's cost per tile a per-CU cost or an aggregate-bandwidth cost?  The
K = 768, N = 768 residual GEMM vs the plain one at growing M: with few tiles (one round on a few
CUs) the difference is the per-tile epilogue cost of an unloaded memory system; at full rounds it
is what the synchronised epilogues of 256 CUs pay.  One JSON line per M."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from mingpt_distributed_amd.ops import gemm as G


def timeit(fn, iters=50, warm=5):
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
    return ts[len(ts) // 2] * 1e3


def main():
    N = K = 768
    r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
    w, b = r(N, K), r(N)
    for M in [256, 768, 2048, 8192, 21760, 43520, 65536, 131072]:
        x, res = r(M, K), r(M, N)
        tiles = -(-M // 256) * 3
        t0 = timeit(lambda: G.gemm_nt(x, w))
        t1 = timeit(lambda: G.gemm_nt(x, w, bias=b, epi="bias"))
        t2 = timeit(lambda: G.gemm_nt(x, w, bias=b, epi="resid", resid=res, p=0.0))
        t3 = timeit(lambda: G.gemm_nt(x, w, bias=b, epi="resid", resid=res, p=0.1, seed=3))
        rounds = -(-tiles // 256)
        print(json.dumps({"M": M, "tiles": tiles, "rounds": rounds, "none_us": round(t0, 1), "bias_us": round(t1, 1),
                          "resid_us": round(t2, 1), "resid_drop_us": round(t3, 1),
                          "resid_extra_per_round_us": round((t2 - t1) / rounds, 2)}), flush=True)


if __name__ == "__main__":
    main()
