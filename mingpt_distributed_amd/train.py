"""Distributed training entrypoint (reference ``/root/reference/mingpt/train.py:11-62``).

    python -m mingpt_distributed_amd.train --config configs/gpt2_config.yaml trainer_config.batch_size=32
    torchrun --standalone --nproc_per_node 8 -m mingpt_distributed_amd.train --config configs/gpt2_124m.yaml

Reads the reference's four-section YAML (Hydra is not installed; ``section.key=value`` and
``--section.key=value`` overrides are both accepted), builds the dataset, splits it, sizes the
model from the data (``vocab_size``/``block_size``), and runs :class:`GPTTrainer`.  The
reference's startup crashes are fixed (D12 ``CharDataset`` signature, D13 missing
``train_split``, D14 ``n_embd`` key).  ``data_config.path: synthetic`` trains on random tokens
(no datasets are downloadable here).
"""
from __future__ import annotations

import argparse
import sys
from typing import List, Optional

import torch
from torch.utils.data import random_split

from .data import CharDataset, DataConfig, SyntheticTokens
from .models import GPT, GPTConfig, OptimizerConfig
from .optim import create_optimizer
from .parallel import dist as D
from .trainer import GPTTrainer
from .utils.config import load_run_config


def get_resources(gpt_config: GPTConfig, optimizer_config: OptimizerConfig, data_config: DataConfig):
    if data_config.path in (None, "synthetic") or str(data_config.path).startswith("synthetic"):
        data = SyntheticTokens(vocab_size=gpt_config.vocab_size or 50257,
                               block_size=data_config.block_size or gpt_config.block_size,
                               size=int(1 << 16))
        vocab = data.vocab_size
    else:
        data = CharDataset(data_config)
        vocab = data.vocab_size
    split = data_config.train_split if data_config.train_split is not None else 0.9
    train_size = int(len(data) * split)
    gen = torch.Generator().manual_seed(0)
    train_set, test_set = random_split(data, [train_size, len(data) - train_size], generator=gen)
    gpt_config.vocab_size = vocab
    gpt_config.block_size = data.block_size
    model = GPT(gpt_config, verbose=D.info().is_main)
    optimizer = create_optimizer(model, optimizer_config)
    return model, optimizer, train_set, test_set


def main(argv: Optional[List[str]] = None) -> GPTTrainer:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--config", default=None, help="four-section YAML (reference gpt2_config.yaml shape)")
    ap.add_argument("--device", default="auto")
    args, overrides = ap.parse_known_args(argv)
    D.init_distributed(device=args.device)
    rc = load_run_config(args.config, overrides)
    torch.manual_seed(rc.trainer_config.seed)
    model, optimizer, train_set, test_set = get_resources(rc.gpt_config, rc.optimizer_config, rc.data_config)
    trainer = GPTTrainer(rc.trainer_config, model, optimizer, train_set, test_set)
    trainer.train()
    D.destroy()
    return trainer


if __name__ == "__main__":
    main(sys.argv[1:])
