#!/usr/bin/env python
"""Loss parity of bf16 vs fp32 gradient reduction (DataParallelEngine ``reduce_dtype``).

``--world`` data-parallel ranks (default 2; 8 = one MI355X node; gloo on CPU, or ``--device cuda``
with every rank on one card) train the
same gpt-mini char-LM from the same init on the same rank-sharded batches, once with fp32 and once
with bf16 gradients on the wire; the per-step losses are written as JSON lines.

    python bench/reduce_dtype_parity.py --steps 200 --out profiles/round2_reduce_dtype_parity.jsonl
    python bench/reduce_dtype_parity.py --world 8 --batch 4 --steps 60 --out profiles/round3_reduce_dtype_parity_8rank_cpu.jsonl
"""
import argparse
import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _text(n=200_000):
    g = torch.Generator().manual_seed(0)
    words = ["the", "quick", "brown", "fox", "jumps", "over", "lazy", "dog", "and", "runs", "far", "away"]
    idx = torch.randint(0, len(words), (n // 5,), generator=g)
    return " ".join(words[i] for i in idx.tolist())[:n]


def _worker(rank, world, port, a, reduce, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from mingpt_distributed_amd.models import GPT, GPTConfig
    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    torch.set_num_threads(max(1, 8 // world))
    D.init_distributed(device=a.device, backend="gloo")
    text = _text()
    chars = sorted(set(text))
    ids = torch.tensor([chars.index(c) for c in text])
    torch.manual_seed(0)
    model = GPT(GPTConfig(model_type="gpt-mini", vocab_size=len(chars), block_size=a.block,
                          embed_drop=0.0, resid_drop=0.0, attn_drop=0.0), verbose=False)
    dev = torch.device("cuda", 0) if a.device == "cuda" else torch.device("cpu")
    eng = StepEngine(model, lr=5e-4, grad_clip=1.0, device=dev, bucket_mb=1.0,
                     reduce_dtype=torch.bfloat16 if reduce == "bf16" else None)
    g = torch.Generator().manual_seed(123)
    losses = []
    for step in range(a.steps):
        starts = torch.randint(0, len(ids) - a.block - 1, (a.batch * world,), generator=g)
        mine = starts[rank * a.batch:(rank + 1) * a.batch]
        x = torch.stack([ids[s:s + a.block] for s in mine]).to(dev)
        y = torch.stack([ids[s + 1:s + a.block + 1] for s in mine]).to(dev)
        loss = eng.train_step([(x, y)])
        losses.append(D.all_reduce_mean(loss.float()).item())
    if rank == 0:
        q.put(losses)
    D.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--block", type=int, default=64)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    res = {}
    for reduce in ("fp32", "bf16"):
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker, args=(r, a.world, port, a, reduce, q)) for r in range(a.world)]
        for p in ps:
            p.start()
        res[reduce] = q.get()
        for p in ps:
            p.join()
    lines = []
    for i in range(a.steps):
        lines.append({"step": i, "loss_fp32": res["fp32"][i], "loss_bf16": res["bf16"][i]})
    k = max(1, a.steps // 10)
    summ = {"summary": True, "device": a.device, "world": a.world, "batch_per_rank": a.batch, "steps": a.steps,
            "final_fp32": sum(res["fp32"][-k:]) / k, "final_bf16": sum(res["bf16"][-k:]) / k,
            "max_abs_diff": max(abs(u - v) for u, v in zip(res["fp32"], res["bf16"]))}
    print(json.dumps(summ))
    if a.out:
        with open(a.out, "w") as f:
            for ln in lines + [summ]:
                f.write(json.dumps(ln) + "\n")


if __name__ == "__main__":
    main()
