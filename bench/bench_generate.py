#!/usr/bin/env python
"""Greedy-decode throughput (BASELINE config #4, the generate.ipynb path) on random GPT-2 124M
weights: this framework's ``GPT.generate`` (prefill once on the gfx950 kernels, then one-token
steps against the KV cache with the decode-attention kernel) vs the reference's algorithm
(``/root/reference/mingpt/model.py:322-356``: re-run the full forward over the whole prefix for
every new token, no cache) in stock PyTorch bf16 (autocast + SDPA).  Prints one JSON line per B."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return out, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompt", type=int, default=32)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--batches", default="1,8")
    a = ap.parse_args()
    from bench.baseline_torch import GPT as TorchGPT
    from mingpt_distributed_amd.models import GPT, GPTConfig

    torch.manual_seed(0)
    ours = GPT(GPTConfig(model_type="gpt2", vocab_size=50257, block_size=1024), verbose=False)
    ours = ours.cuda().to(torch.bfloat16).eval()
    ref = TorchGPT(p=0.0, attn="sdpa").cuda().eval()
    for B in map(int, a.batches.split(",")):
        idx = torch.randint(0, 50257, (B, a.prompt), device="cuda")
        with torch.no_grad():
            ours.generate(idx, 4, do_sample=False)  # warm-up (kernels, caches)
            out, t_ours = timed(lambda: ours.generate(idx, a.new, do_sample=False))

            def ref_generate():
                x = idx
                for _ in range(a.new):
                    with torch.autocast("cuda", dtype=torch.bfloat16):
                        logits, _ = ref(x[:, -1024:])
                    x = torch.cat([x, logits[:, -1, :].argmax(-1, keepdim=True)], dim=1)
                return x
            ref_generate() if a.new <= 8 else None
            _, t_ref = timed(ref_generate)
        assert out.shape == (B, a.prompt + a.new)
        print(json.dumps({"metric": "greedy decode tokens/s", "model": "gpt2 (random init)", "batch": B,
                          "prompt": a.prompt, "new_tokens": a.new,
                          "ours_kv_cache_tok_s": round(B * a.new / t_ours, 1),
                          "reference_algorithm_torch_tok_s": round(B * a.new / t_ref, 1),
                          "speedup": round(t_ref / t_ours, 2)}), flush=True)


if __name__ == "__main__":
    main()
