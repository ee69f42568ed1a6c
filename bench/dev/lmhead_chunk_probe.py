#!/usr/bin/env python
"""Does a row chunk of the LM-head logits stay in the MI355X's 256 MB Infinity Cache between the
GEMM that writes it and the cross-entropy pass that reads it?  Full-batch GEMM + xent_fused vs the
same work in row chunks (each chunk's logits ~CH x 50304 x 2 B), timing the GEMMs and the xent
passes separately (CUDA events around each launch).  One JSON line per chunk size."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext


def main():
    C = ext()
    M, D, V = 131072, 768, 50257
    ld = (V + 127) // 128 * 128
    h = (torch.randn(M, D, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(V, D, device="cuda") * 0.02).to(torch.bfloat16)
    t = torch.randint(0, V, (M,), device="cuda")
    for CH in [131072, 16384, 4096, 2048, 1280]:
        ev = []
        for rep in range(3):
            tg = tx = 0.0
            for r0 in range(0, M, CH):
                r1 = min(M, r0 + CH)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                lg = G.gemm_nt(h[r0:r1], w, ld=ld)
                e[1].record()
                out = C.xent_fused(lg, t[r0:r1], V)
                e[2].record()
                ev.append(e)
                del lg, out
            torch.cuda.synchronize()
        n = (M + CH - 1) // CH
        last = ev[-n:]
        tg = sum(a.elapsed_time(b) for a, b, _ in last)
        tx = sum(b.elapsed_time(c) for _, b, c in last)
        print(json.dumps({"chunk_rows": CH, "chunk_logits_MB": round(CH * ld * 2 / 1e6), "chunks": n,
                          "gemm_ms": round(tg, 3), "xent_ms": round(tx, 3), "total_ms": round(tg + tx, 3)}), flush=True)


if __name__ == "__main__":
    main()
