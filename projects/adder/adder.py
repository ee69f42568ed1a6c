#!/usr/bin/env python
"""Train a GPT to add n-digit numbers (upstream ``projects/adder``, README ``/root/reference/README.md:12``).

    python projects/adder/adder.py --trainer.max_iters=3000
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
from torch.utils.data.dataloader import DataLoader

from mingpt_distributed_amd.data import AdditionDataset
from mingpt_distributed_amd.models import GPT
from mingpt_distributed_amd.trainer import Trainer
from mingpt_distributed_amd.utils import CfgNode as CN
from mingpt_distributed_amd.utils import set_seed, setup_logging


def get_config():
    C = CN()
    C.system = CN()
    C.system.seed = 3407
    C.system.work_dir = "./out/adder"
    C.data = CN()
    C.data.ndigit = 2
    C.model = GPT.get_default_config()
    C.model.model_type = "gpt-nano"
    C.trainer = Trainer.get_default_config()
    C.trainer.learning_rate = 5e-4
    C.trainer.max_iters = 5000
    C.trainer.num_workers = 0
    return C


def eval_split(model, dataset, device, max_batches=None):
    nd = dataset.ndigit
    loader = DataLoader(dataset, batch_size=100, num_workers=0, drop_last=False)
    results = []
    factors = torch.tensor([[10 ** i for i in range(nd + 1)][::-1]], device=device)
    for b, (x, y) in enumerate(loader):
        x = x.to(device)
        d1d2 = x[:, : nd * 2]
        d1d2d3 = model.generate(d1d2, nd + 1, do_sample=False)
        d3 = d1d2d3[:, -(nd + 1):].flip(1)
        d1i = (d1d2[:, :nd] * factors[:, 1:]).sum(1)
        d2i = (d1d2[:, nd: nd * 2] * factors[:, 1:]).sum(1)
        d3i_pred = (d3 * factors).sum(1)
        results.extend((d3i_pred == d1i + d2i).cpu().tolist())
        if max_batches is not None and b + 1 >= max_batches:
            break
    return sum(results) / max(1, len(results))


def main(argv):
    config = get_config()
    config.merge_from_args(argv)
    set_seed(config.system.seed)
    setup_logging(config)
    train_dataset = AdditionDataset("train", config.data.ndigit)
    test_dataset = AdditionDataset("test", config.data.ndigit)
    config.model.vocab_size = train_dataset.get_vocab_size()
    config.model.block_size = train_dataset.get_block_size()
    model = GPT(config.model)
    trainer = Trainer(config.trainer, model, train_dataset)

    def batch_end_callback(trainer):
        if trainer.iter_num % 10 == 0:
            print(f"iter_dt {trainer.iter_dt * 1000:.2f}ms; iter {trainer.iter_num}: train loss {trainer.loss.item():.5f}")
        if trainer.iter_num % 500 == 0:
            model.eval()
            with torch.no_grad():
                acc = eval_split(model, test_dataset, trainer.engine.device, max_batches=5)
            print(f"test accuracy {acc:.3f}")
            model.train()

    trainer.set_callback("on_batch_end", batch_end_callback)
    trainer.run()
    return trainer


if __name__ == "__main__":
    main(sys.argv[1:])
