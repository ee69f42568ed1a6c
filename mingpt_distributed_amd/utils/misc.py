"""Small utilities: seeding, run-dir logging, model-size print.

``print_model_size`` mirrors ``/root/reference/mingpt/model.py:21-33``; ``set_seed`` and
``setup_logging`` are the upstream-minGPT utilities the reference README advertises
(``/root/reference/README.md:27-54``).
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np
import torch


def set_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def setup_logging(config) -> None:
    """Create ``config.system.work_dir`` and dump args + config there (upstream behaviour)."""
    work_dir = config.system.work_dir
    os.makedirs(work_dir, exist_ok=True)
    with open(os.path.join(work_dir, "args.txt"), "w") as f:
        f.write(" ".join(sys.argv))
    with open(os.path.join(work_dir, "config.json"), "w") as f:
        f.write(json.dumps(config.to_dict(), indent=4, default=str))


def model_size_bytes(model: torch.nn.Module) -> int:
    n = sum(p.numel() * p.element_size() for p in model.parameters())
    n += sum(b.numel() * b.element_size() for b in model.buffers())
    return n


def print_model_size(model: torch.nn.Module) -> float:
    """Print params+buffers size in MB and return it (reference ``model.py:21-33``)."""
    mb = model_size_bytes(model) / 1024 ** 2
    print(f"Model size (MB): {mb:.3f}")
    return mb
