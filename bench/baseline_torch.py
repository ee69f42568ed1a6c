#!/usr/bin/env python
"""Self-baseline: the reference's training step as plain PyTorch-ROCm eager + torch DDP.

The reference publishes no numbers, so the number to beat is the reference's
own algorithm run on the same MI355X: a minGPT GPT-2 (canonical architecture, the reference's
bugs fixed: causal -inf mask, GELU between the MLP linears), ``torch.autocast(bf16)``,
``torch.optim.AdamW``, ``clip_grad_norm_``, wrapped in ``DistributedDataParallel`` over the
``nccl`` (=RCCL) backend exactly as ``/root/reference/mingpt/trainer.py:71,118-133`` does.
Attention is either the upstream explicit masked softmax (``--attn math``, what minGPT runs)
or torch SDPA (``--attn sdpa``, the strongest stock-PyTorch option) -- both are reported.

Usage: ``python bench/baseline_torch.py --batch 16 --steps 10 --warmup 3 [--attn sdpa]``
(or under torchrun for N GPUs).  Prints one JSON line from rank 0.
"""
import argparse
import json
import math
import os
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class CausalSelfAttention(nn.Module):
    def __init__(self, D, H, T, p, attn):
        super().__init__()
        self.c_attn = nn.Linear(D, 3 * D)
        self.c_proj = nn.Linear(D, D)
        self.attn_drop = nn.Dropout(p)
        self.resid_drop = nn.Dropout(p)
        self.H, self.attn, self.p = H, attn, p
        self.register_buffer("bias", torch.tril(torch.ones(T, T)).view(1, 1, T, T), persistent=False)

    def forward(self, x):
        B, T, C = x.shape
        q, k, v = self.c_attn(x).split(C, dim=2)
        q, k, v = (t.view(B, T, self.H, C // self.H).transpose(1, 2) for t in (q, k, v))
        if self.attn == "sdpa":
            y = F.scaled_dot_product_attention(q, k, v, dropout_p=self.p if self.training else 0.0,
                                               is_causal=True)
        else:
            att = (q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(k.size(-1)))
            att = att.masked_fill(self.bias[:, :, :T, :T] == 0, float("-inf"))
            att = self.attn_drop(F.softmax(att, dim=-1))
            y = att @ v
        y = y.transpose(1, 2).contiguous().view(B, T, C)
        return self.resid_drop(self.c_proj(y))


class Block(nn.Module):
    def __init__(self, D, H, T, p, attn):
        super().__init__()
        self.ln_1 = nn.LayerNorm(D)
        self.attn = CausalSelfAttention(D, H, T, p, attn)
        self.ln_2 = nn.LayerNorm(D)
        self.mlp = nn.Sequential(nn.Linear(D, 4 * D), nn.GELU(approximate="tanh"), nn.Linear(4 * D, D),
                                 nn.Dropout(p))

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class GPT(nn.Module):
    def __init__(self, V=50257, T=1024, L=12, H=12, D=768, p=0.1, attn="math"):
        super().__init__()
        self.wte, self.wpe = nn.Embedding(V, D), nn.Embedding(T, D)
        self.drop = nn.Dropout(p)
        self.h = nn.ModuleList([Block(D, H, T, p, attn) for _ in range(L)])
        self.ln_f = nn.LayerNorm(D)
        self.lm_head = nn.Linear(D, V, bias=False)
        self.lm_head.weight = self.wte.weight  # GPT-2 weight tying
        for n, prm in self.named_parameters():
            if prm.dim() >= 2:
                nn.init.normal_(prm, 0.0, 0.02 / math.sqrt(2 * L) if n.endswith("c_proj.weight") else 0.02)

    def forward(self, idx, targets=None):
        T = idx.size(1)
        x = self.drop(self.wte(idx) + self.wpe(torch.arange(T, device=idx.device)))
        for b in self.h:
            x = b(x)
        logits = self.lm_head(self.ln_f(x))
        if targets is None:
            return logits, None
        return logits, F.cross_entropy(logits.view(-1, logits.size(-1)), targets.view(-1), ignore_index=-1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--attn", default="math", choices=["math", "sdpa"])
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--vocab", type=int, default=50257)
    a = ap.parse_args()
    dims = {"gpt2": (12, 12, 768), "gpt2-xl": (48, 25, 1600), "gpt2-medium": (24, 16, 1024),
            "gpt-mini": (6, 6, 192)}[a.model]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        torch.distributed.init_process_group("nccl")
    torch.manual_seed(0)
    model = GPT(V=a.vocab, T=a.seq, L=dims[0], H=dims[1], D=dims[2], p=a.dropout, attn=a.attn).cuda()
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1)
    x = torch.randint(0, a.vocab, (a.batch, a.seq), device="cuda")
    y = torch.randint(0, a.vocab, (a.batch, a.seq), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, loss = model(x, y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    tok = a.batch * a.seq * a.steps * world / dt
    if rank == 0:
        print(json.dumps({"metric": "baseline_torch_eager_tokens_per_s", "value": tok, "n_gpus": world,
                          "ms_per_step": dt / a.steps * 1e3, "batch_per_gpu": a.batch, "seq": a.seq,
                          "attn": a.attn, "dropout": a.dropout, "model": a.model, "vocab": a.vocab,
                          "loss": float(loss.item()),
                          "max_mem_gb": torch.cuda.max_memory_allocated() / 2**30}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
