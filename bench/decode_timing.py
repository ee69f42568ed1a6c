#!/usr/bin/env python
"""Greedy decode throughput of GPT.generate for an fp32-loaded model (the generate.ipynb /
projects/generate path: weights left fp32, bf16 copies made once by the decode path) and a bf16
model, GPT-2 124M random init, B = 1 and 8.  One JSON line per (dtype, B)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig

new = int(os.environ.get("NEW", "256"))
torch.manual_seed(0)
base = GPT(GPTConfig(model_type="gpt2", vocab_size=50257, block_size=1024), verbose=False).eval()
for dt in (torch.float32, torch.bfloat16):
    m = GPT(GPTConfig(model_type="gpt2", vocab_size=50257, block_size=1024), verbose=False).eval()
    m.load_state_dict(base.state_dict())
    m = m.cuda().to(dt)
    for B in (1, 8):
        idx = torch.randint(0, 50257, (B, 32), device="cuda")
        with torch.no_grad():
            m.generate(idx, 8, do_sample=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = m.generate(idx, new, do_sample=False)
            torch.cuda.synchronize()
            dt_s = time.perf_counter() - t0
        print(json.dumps({"weights": str(dt).split(".")[-1], "batch": B, "new_tokens": new,
                          "tok_s": round(B * new / dt_s, 1), "ms_per_step": round(dt_s / new * 1e3, 3)}), flush=True)
