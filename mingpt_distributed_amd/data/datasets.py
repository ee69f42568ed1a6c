"""Toy and synthetic datasets.

* :class:`SortDataset` -- the ``demo.ipynb`` task advertised by the reference README
  (``/root/reference/README.md:14``): sort ``length`` digits in ``[0, num_digits)``; inputs are the
  unsorted digits followed by the sorted prefix, targets mask the prompt part with -1.  A fixed
  1-in-4 hash of each example assigns it to train/test.
* :class:`AdditionDataset` -- ``projects/adder`` (``README.md:12``): ``a + b = c`` with ``ndigit``
  digit operands, ``c`` rendered reversed; targets for the operand digits are -1.
* :class:`SyntheticTokens` -- random token sequences of a given vocab/length, deterministic per
  index: the stand-in for GPT-2 pre-training data (no datasets are downloadable here).
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


class SortDataset(Dataset):
    def __init__(self, split: str, length: int = 6, num_digits: int = 3, size: int = 10000, seed: int = 0):
        assert split in {"train", "test"}
        self.split, self.length, self.num_digits = split, length, num_digits
        self.size, self.seed = size, seed

    def get_vocab_size(self) -> int:
        return self.num_digits

    def get_block_size(self) -> int:
        return self.length * 2 - 1

    def __len__(self) -> int:
        return self.size

    def _split_of(self, inp) -> str:
        h = 0
        for d in inp.tolist():
            h = (h * 1000003 + d + 1) & 0xFFFFFFFF
        return "test" if h % 4 == 0 else "train"

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 7919 + idx * 2 + (self.split == "test"))
        while True:
            inp = torch.randint(self.num_digits, size=(self.length,), generator=g, dtype=torch.long)
            # half the time, insist on many repeated digits (harder cases), as upstream does
            if torch.rand(1, generator=g).item() < 0.5 and inp.unique().numel() > self.length // 2:
                continue
            if self._split_of(inp) == self.split:
                break
        sol = torch.sort(inp)[0]
        cat = torch.cat((inp, sol), dim=0)
        x = cat[:-1].clone()
        y = cat[1:].clone()
        y[: self.length - 1] = -1
        return x, y


class AdditionDataset(Dataset):
    def __init__(self, split: str, ndigit: int = 2):
        assert split in {"train", "test"}
        self.ndigit = ndigit
        num = (10 ** ndigit) ** 2
        rng = torch.Generator().manual_seed(1337)
        perm = torch.randperm(num, generator=rng)
        num_test = min(int(num * 0.2), 500)
        self.ixes = perm[:num_test] if split == "test" else perm[num_test:]

    def get_vocab_size(self) -> int:
        return 10

    def get_block_size(self) -> int:
        return 3 * self.ndigit + 1 - 1

    def __len__(self) -> int:
        return self.ixes.nelement()

    def __getitem__(self, idx):
        nd = self.ndigit
        i = self.ixes[idx].item()
        a, b = divmod(i, 10 ** nd)
        c = a + b
        render = f"{a:0{nd}d}{b:0{nd}d}" + f"{c:0{nd + 1}d}"[::-1]
        dix = [int(s) for s in render]
        x = torch.tensor(dix[:-1], dtype=torch.long)
        y = torch.tensor(dix[1:], dtype=torch.long)
        y[: nd * 2 - 1] = -1
        return x, y


class SyntheticTokens(Dataset):
    def __init__(self, vocab_size: int = 50257, block_size: int = 1024, size: int = 1 << 20, seed: int = 0):
        self.vocab_size, self.block_size, self.size, self.seed = vocab_size, block_size, size, seed

    def get_vocab_size(self) -> int:
        return self.vocab_size

    def get_block_size(self) -> int:
        return self.block_size

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        seq = torch.randint(self.vocab_size, (self.block_size + 1,), generator=g)
        return seq[:-1], seq[1:]
