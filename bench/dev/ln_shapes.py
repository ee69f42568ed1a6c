#!/usr/bin/env python
"""LayerNorm kernels in isolation at the GPT-2 (D = 768) and gpt2-xl (D = 1600) step shapes: time and
effective HBM bandwidth of the forward, the plain backward (+ residual gradient) and the backward
with the fused residual-dropout hand-off (layernorm.hip).  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from mingpt_distributed_amd.ops._ext import ext


def timeit(fn, iters=30, warm=5):
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
    C = ext()
    for M, D in [(131072, 768), (16384, 1600), (32768, 1600), (65536, 1600)]:
        r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)
        x, w, b, dy, dres = r(M, D), r(D), r(D), r(M, D), r(M, D)
        y, mean, rstd = C.layernorm_fwd(x, w, b, 1e-5)
        dw, db, dzb = (torch.zeros(D, device="cuda") for _ in range(3))
        tf = timeit(lambda: C.layernorm_fwd(x, w, b, 1e-5))
        tb = timeit(lambda: C.layernorm_bwd(dy, x, w, mean, rstd, dw, db, dres))
        td = timeit(lambda: C.layernorm_bwd_dropout(dy, x, w, mean, rstd, dw, db, dres, dzb, 0.1, 7))
        pl = M * D * 2 / 1e3  # one bf16 plane in GB/s-per-us units (bytes / 1e3 -> GB/s with us)
        print(json.dumps({"M": M, "D": D, "fwd_us": round(tf, 1), "fwd_TBps": round(2 * pl / tf / 1e3, 2),
                          "bwd_us": round(tb, 1), "bwd_TBps": round(4 * pl / tb / 1e3, 2),
                          "bwd_drop_us": round(td, 1), "bwd_drop_TBps": round(5 * pl / td / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
