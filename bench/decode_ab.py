#!/usr/bin/env python
"""Greedy decode tokens/s of GPT.generate alone (GPT-2 124M random init, bf16, 32-token prompt,
NEW new tokens), best of REPS timed runs per batch: the quick form of bench_generate.py for
one-box A/Bs of decode-kernel switches (each variant in its own process).  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig

new, reps = int(os.environ.get("NEW", "256")), int(os.environ.get("REPS", "3"))
torch.manual_seed(0)
m = GPT(GPTConfig(model_type="gpt2", vocab_size=50257, block_size=1024), verbose=False)
m = m.cuda().to(torch.bfloat16).eval()
res = {"variant": os.environ.get("VARIANT", "")}
for B in (1, 8):
    idx = torch.randint(0, 50257, (B, 32), device="cuda")
    best = 0.0
    with torch.no_grad():
        m.generate(idx, 8, do_sample=False)
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.generate(idx, new, do_sample=False)
            torch.cuda.synchronize()
            best = max(best, B * new / (time.perf_counter() - t0))
    res[f"B{B}_tok_s"] = round(best, 1)
print(json.dumps(res), flush=True)
