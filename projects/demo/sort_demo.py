#!/usr/bin/env python
"""Sort-task demo (upstream minGPT ``demo.ipynb``, advertised by ``/root/reference/README.md:13``).

Trains ``gpt-nano`` to sort sequences of 6 digits from {0,1,2}, then scores exact-match accuracy
on held-out sequences with greedy generation.  Runs on CPU in about a minute, or on a GPU through
the fused gfx950 kernels (``--device cuda``).

    python projects/demo/sort_demo.py [--device cpu|cuda] [--iters 2000]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from mingpt_distributed_amd.data import SortDataset
from mingpt_distributed_amd.models import GPT
from mingpt_distributed_amd.trainer import Trainer
from mingpt_distributed_amd.utils import set_seed


@torch.no_grad()
def eval_split(model, dataset, device, max_batches=None, batch_size=100):
    """Exact-match accuracy of greedy sorting (upstream ``eval_split``)."""
    n = dataset.length
    loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, num_workers=0, drop_last=False)
    correct, total = 0, 0
    for b, (x, y) in enumerate(loader):
        x = x.to(device)
        inp = x[:, :n]
        sol = y[:, -n:].to(device)
        cat = model.generate(inp, n, do_sample=False)
        pred = cat[:, n:]
        correct += (pred == sol).all(1).sum().item()
        total += x.size(0)
        if max_batches is not None and b + 1 >= max_batches:
            break
    return correct / max(total, 1)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="auto")
    ap.add_argument("--iters", type=int, default=2000)
    a = ap.parse_args(argv)
    set_seed(3407)
    train, test = SortDataset("train"), SortDataset("test")
    C = GPT.get_default_config()
    C.model_type = "gpt-nano"
    C.vocab_size = train.get_vocab_size()
    C.block_size = train.get_block_size()
    model = GPT(C)
    tc = Trainer.get_default_config()
    tc.learning_rate = 5e-4
    tc.max_iters = a.iters
    tc.num_workers = 0
    tc.device = a.device
    trainer = Trainer(tc, model, train)

    def log(t):
        if t.iter_num % 100 == 0:
            print(f"iter_dt {t.iter_dt * 1000:.2f}ms; iter {t.iter_num}: train loss {t.loss.item():.5f}")

    trainer.set_callback("on_batch_end", log)
    trainer.run()
    model.eval()
    dev = trainer.engine.device
    tr_acc = eval_split(model, train, dev, max_batches=50)
    te_acc = eval_split(model, test, dev, max_batches=50)
    print(f"train exact-match {tr_acc:.4f}  test exact-match {te_acc:.4f}")
    return tr_acc, te_acc


if __name__ == "__main__":
    main()
