#!/usr/bin/env python
"""Prompted text generation from a GPT-2 checkpoint (upstream ``generate.ipynb``, advertised by
``/root/reference/README.md:15``).

No network here: point ``--weights`` at a local GPT-2 checkpoint (HF ``model.safetensors`` /
``pytorch_model.bin`` directory, loaded with safe loaders) and ``MINGPT_BPE_DIR`` at a directory
holding ``encoder.json`` + ``vocab.bpe``.  ``--random-init`` runs the same path on random weights
(for smoke tests; the text is noise).  On a GPU the prompt is prefilled once and every new token
is one fused-kernel decode step against the KV cache.

    python projects/generate/generate.py --weights /path/to/gpt2 --prompt "Andrej Karpathy, the" \
        --num-samples 5 --steps 20 --device cuda
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.utils import set_seed


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model-type", default="gpt2")
    ap.add_argument("--weights", default=None, help="local GPT-2 checkpoint (file or HF directory)")
    ap.add_argument("--random-init", action="store_true")
    ap.add_argument("--prompt", default="")
    ap.add_argument("--num-samples", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top-k", type=int, default=40)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--greedy", action="store_true")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--seed", type=int, default=3407)
    a = ap.parse_args(argv)
    dev = a.device if a.device != "auto" else ("cuda" if torch.cuda.is_available() else "cpu")
    set_seed(a.seed)
    if a.random_init:
        model = GPT(GPTConfig(model_type=a.model_type, vocab_size=50257, block_size=1024), verbose=False)
    else:
        model = GPT.from_pretrained(a.model_type, source=a.weights)
    model.to(dev).eval()

    tok = None
    try:
        from mingpt_distributed_amd.bpe import BPETokenizer

        tok = BPETokenizer()
    except Exception as e:  # vocab files absent: fall back to raw token ids
        print(f"(no BPE vocabulary available: {e}; printing token ids)")
    if tok is not None:
        x = tok(a.prompt if a.prompt else "<|endoftext|>").to(dev) if a.prompt else \
            torch.tensor([[50256]], dtype=torch.long, device=dev)
    else:
        x = torch.tensor([[50256]], dtype=torch.long, device=dev)
    x = x.expand(a.num_samples, -1).contiguous()
    y = model.generate(x, max_new_tokens=a.steps, temperature=a.temperature, do_sample=not a.greedy,
                       top_k=a.top_k)
    outs = []
    for i in range(a.num_samples):
        out = tok.decode(y[i].cpu().squeeze()) if tok is not None else y[i].tolist()
        outs.append(out)
        print("-" * 80)
        print(out)
    return outs


if __name__ == "__main__":
    main()
