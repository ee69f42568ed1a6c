#!/usr/bin/env python
"""Character-level GPT on a text file (upstream ``projects/chargpt``, advertised by the reference
README ``/root/reference/README.md:13``; BASELINE.json config #2: gpt-mini, bf16, 1 MI355X).

    python projects/chargpt/chargpt.py --data.path=input.txt --trainer.max_iters=2000
Overrides use the CfgNode ``--section.key=value`` form.  With no input file, a synthetic
corpus is generated (there is no network to fetch tiny-shakespeare).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from mingpt_distributed_amd.data import CharDataset
from mingpt_distributed_amd.models import GPT
from mingpt_distributed_amd.trainer import Trainer
from mingpt_distributed_amd.utils import CfgNode as CN
from mingpt_distributed_amd.utils import set_seed, setup_logging


def get_config():
    C = CN()
    C.system = CN()
    C.system.seed = 3407
    C.system.work_dir = "./out/chargpt"
    C.data = CN()
    C.data.path = "input.txt"
    C.data.block_size = 128
    C.model = GPT.get_default_config()
    C.model.model_type = "gpt-mini"
    C.trainer = Trainer.get_default_config()
    C.trainer.learning_rate = 5e-4
    C.trainer.max_iters = 2000
    C.trainer.num_workers = 0
    C.trainer.cuda_graph = True  # gpt-mini at T=128 is launch-bound: one hipGraph replay per step
    C.sample_every = 500
    return C


def synthetic_corpus(n=200_000, seed=0):
    g = torch.Generator().manual_seed(seed)
    words = ["the", "king", "queen", "lord", "god", "love", "death", "night", "day", "heart", "O", "my",
             "thou", "art", "and", "to", "of", "in", "is", "not", "with", "fair", "sweet", "blood"]
    out, k = [], 0
    while k < n:
        line = " ".join(words[i] for i in torch.randint(len(words), (8,), generator=g).tolist())
        out.append(line.capitalize() + ".\n")
        k += len(out[-1])
    return "".join(out)


def main(argv):
    config = get_config()
    config.merge_from_args(argv)
    set_seed(config.system.seed)
    setup_logging(config)
    if os.path.exists(config.data.path):
        text = open(config.data.path, "r").read()
    else:
        print(f"{config.data.path} not found: using a synthetic corpus")
        text = synthetic_corpus()
    train_dataset = CharDataset(config.data, text)
    config.model.vocab_size = train_dataset.get_vocab_size()
    config.model.block_size = train_dataset.get_block_size()
    model = GPT(config.model)
    trainer = Trainer(config.trainer, model, train_dataset)

    def batch_end_callback(trainer):
        if trainer.iter_num % 10 == 0:
            print(f"iter_dt {trainer.iter_dt * 1000:.2f}ms; iter {trainer.iter_num}: train loss {trainer.loss.item():.5f}")
        if trainer.iter_num % config.sample_every == 0:
            model.eval()
            with torch.no_grad():
                context = "O God, O God!"
                context = "".join(c for c in context if c in train_dataset.stoi) or text[:8]
                x = train_dataset.encode(context)[None].to(trainer.engine.device)
                y = model.generate(x, 500, temperature=1.0, do_sample=True, top_k=10)[0]
                print(train_dataset.decode(y))
            torch.save(model.state_dict(), os.path.join(config.system.work_dir, "model.pt"))
            model.train()

    trainer.set_callback("on_batch_end", batch_end_callback)
    trainer.run()
    return trainer


if __name__ == "__main__":
    main(sys.argv[1:])
