"""Per-rank HBM of replicated DP vs ZeRO-1 (parallel/zero.py) on one card: 2 ranks over gloo.

Not a throughput bench (gloo stages the collectives through host memory); it measures what
ZeRO-1 is for: optimizer-state bytes and peak allocated memory per rank.
    python bench/bench_zero_mem.py [--model gpt2-medium] [--batch 4]
"""
import argparse
import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(rank, world, port, a, zero1, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from mingpt_distributed_amd.models import GPT, GPTConfig
    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    D.init_distributed(device="cuda", backend="gloo")
    torch.manual_seed(0)
    model = GPT(GPTConfig(model_type=a.model, vocab_size=50257, block_size=1024), verbose=False)
    eng = StepEngine(model, device=torch.device("cuda", 0), zero1=zero1)
    x = torch.randint(0, 50257, (a.batch, 1024), device="cuda")
    for _ in range(2):
        loss = eng.train_step([(x, x)])
    torch.cuda.synchronize()
    opt_bytes = (eng.opt.exp_avg.numel() + eng.opt.exp_avg_sq.numel()) * 4
    peak_train = torch.cuda.max_memory_allocated()
    # snapshot cost: what a checkpoint adds on the device on top of training's resident state
    # (ZeRO-1 consolidate() gathers the moments into rank-0 HOST memory, one bucket at a time)
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    if hasattr(eng.opt, "consolidate"):
        eng.opt.consolidate()
    if rank == 0:
        sd = eng.opt.state_dict()
        del sd
    torch.cuda.synchronize()
    q.put({"rank": rank, "zero1": zero1, "loss": float(loss), "opt_state_gb": opt_bytes / 1e9,
           "max_alloc_gb": peak_train / 1e9,
           "snapshot_extra_gb": (torch.cuda.max_memory_allocated() - base) / 1e9})
    D.destroy()


def run(a, zero1):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, a, zero1, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return sorted(out, key=lambda r: r["rank"])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    for z in (False, True):
        for r in run(a, z):
            print(json.dumps(dict(r, model=a.model, batch=a.batch)), flush=True)
