#!/usr/bin/env python
"""Flagship benchmark: GPT-2 124M, seq 1024, bf16 training throughput (tokens/s, whole node).

Metric/config are the ones BASELINE.json names.  One process per GPU (torchrun env), data
parallel over RCCL.  Synthetic random-token batches of the exact training shape and random-init
weights (no datasets or checkpoints are reachable); every timed step is a full training step:
forward, backward, bucketed all-reduce, global grad-norm clip and fused AdamW update, with the
reference's dropout (0.1) active.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model gpt2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

W untimed warmup steps, then K steps bracketed by barrier + device sync; the max over ranks is
reported.  ``vs_baseline`` divides by N x the measured single-GPU torch-eager self-baseline of the
same step at the same per-GPU batch, i.e. the per-GPU speedup over stock
PyTorch-ROCm (the reference publishes no numbers).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch

# single-GPU torch-eager self-baseline at the SAME per-GPU batch, model, shape and dropout
# (bench/baseline_torch.py: torch.autocast bf16, SDPA attention, torch AdamW, MI355X):
# BASELINE.md "Self-baseline" table.
BASELINE_TOK_S_PER_GPU = {16: 367595.5, 32: 413092.9, 64: 461947.8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64,
                    help="sequences per GPU per step (64 x 1024 tokens: ~36 GB of the 288 GB HBM)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--vocab", type=int, default=50257, help="65 = chargpt's character vocabulary")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--zero1", action="store_true",
                    help="shard the AdamW state over the ranks (reduce-scatter + all-gather)")
    ap.add_argument("--profile", default="", help="write a torch.profiler trace to this dir")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as one hipGraph (single GPU; StepEngine.graph_step)")
    a = ap.parse_args()

    from mingpt_distributed_amd.models import GPT, GPTConfig
    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    info = D.init_distributed(device="cuda")
    if info.world_size != a.gpus:
        if info.rank == 0:
            print(f"warning: --gpus {a.gpus} but WORLD_SIZE={info.world_size}; using WORLD_SIZE",
                  file=sys.stderr)
    N = info.world_size
    torch.manual_seed(1234 + info.rank)
    cfg = GPTConfig(model_type=a.model, vocab_size=a.vocab, block_size=a.seq, embed_drop=a.dropout,
                    resid_drop=a.dropout, attn_drop=a.dropout)
    torch.manual_seed(1234)  # identical init on every rank (the engine also broadcasts rank 0)
    model = GPT(cfg, verbose=info.rank == 0)
    eng = StepEngine(model, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, grad_clip=1.0,
                     bucket_mb=a.bucket_mb, zero1=a.zero1)
    g = torch.Generator(device=eng.device).manual_seed(99 + info.rank)
    nb = 4
    xs = [torch.randint(0, a.vocab, (a.batch, a.seq), device=eng.device, generator=g) for _ in range(nb)]
    ys = [torch.randint(0, a.vocab, (a.batch, a.seq), device=eng.device, generator=g) for _ in range(nb)]

    step = (lambda x, y: eng.graph_step(x, y)) if a.graph else (lambda x, y: eng.train_step([(x, y)]))
    for i in range(a.warmup):
        loss = step(xs[i % nb], ys[i % nb])
    D.barrier()
    torch.cuda.synchronize()
    prof = None
    if a.profile and info.rank == 0:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(xs[i % nb], ys[i % nb])
    torch.cuda.synchronize()
    D.barrier()
    dt = time.perf_counter() - t0
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(a.profile, exist_ok=True)
        prof.export_chrome_trace(os.path.join(a.profile, "trace.json"))
        with open(os.path.join(a.profile, "summary.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    dt = D.all_reduce_max(dt, eng.device)
    loss_v = D.all_reduce_mean(loss.float()).item()
    tokens = a.batch * a.seq * a.steps * N
    value = tokens / dt
    if info.rank == 0:
        out = {
            "metric": "tokens/sec (whole node), GPT-2 124M seq1024 bf16" if a.model == "gpt2"
            else f"tokens/sec (whole node), {a.model} seq{a.seq} vocab{a.vocab} bf16",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (BASELINE_TOK_S_PER_GPU[a.batch] * N), 3)
            if a.model == "gpt2" and a.seq == 1024 and a.vocab == 50257 and a.batch in BASELINE_TOK_S_PER_GPU
            else None,
            "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)",
            "config": {"model": a.model, "global_batch": a.batch * N, "seq_len": a.seq,
                       "parallelism": f"dp{N}" + ("-zero1" if eng.zero1 else ""), "micro_batch_per_gpu": a.batch, "dropout": a.dropout,
                       "bucket_mb": a.bucket_mb, "hip_graph": bool(a.graph and N == 1)},
            "loss": round(loss_v, 4),
            "max_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2),
        }
        print(json.dumps(out), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
