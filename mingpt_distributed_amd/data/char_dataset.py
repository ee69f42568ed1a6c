"""Character-level dataset (reference ``/root/reference/mingpt/char_dataset.py:12-47``).

``CharDataset(DataConfig)`` reads ``config.path`` through fsspec (local, ``memory://``, or any
fsspec URL), truncates to ``config.truncate`` of the text, builds ``stoi``/``itos`` over the sorted
unique characters, and serves ``(x = ids[i:i+T], y = ids[i+1:i+T+1])`` as int64.  The upstream
chargpt form ``CharDataset(config, data)`` (text passed in, ``get_vocab_size()``/
``get_block_size()``) is accepted too.  The text is encoded once into a compact tensor (the
reference re-encodes every window in Python on every ``__getitem__``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
from torch.utils.data import Dataset


@dataclass
class DataConfig:
    path: Optional[str] = None
    block_size: Optional[int] = None
    train_split: Optional[float] = 0.9  # reference YAML omits it (D13); default to 90/10
    truncate: float = 1.0


class CharDataset(Dataset):
    def __init__(self, config, data: Optional[str] = None, verbose: bool = True):
        if data is None:
            import fsspec

            with fsspec.open(config.path, "r") as f:
                data = f.read()
        truncate = getattr(config, "truncate", 1.0) or 1.0
        data = data[: int(len(data) * truncate)]
        chars = sorted(set(data))
        if verbose:
            print(f"Data has {len(data)} characters, {len(chars)} unique.")
        self.stoi = {ch: i for i, ch in enumerate(chars)}
        self.itos = {i: ch for i, ch in enumerate(chars)}
        self.block_size = config.block_size
        self.vocab_size = len(chars)
        self.data = data
        dtype = torch.uint8 if len(chars) <= 256 else torch.int32
        self.ids = torch.tensor([self.stoi[c] for c in data], dtype=dtype)
        if len(self.ids) <= self.block_size:
            raise ValueError("text is shorter than block_size + 1")

    def get_vocab_size(self) -> int:
        return self.vocab_size

    def get_block_size(self) -> int:
        return self.block_size

    def encode(self, s: str) -> torch.Tensor:
        return torch.tensor([self.stoi[c] for c in s], dtype=torch.long)

    def decode(self, ids) -> str:
        return "".join(self.itos[int(i)] for i in ids)

    def __len__(self) -> int:
        return len(self.ids) - self.block_size

    def __getitem__(self, idx):
        chunk = self.ids[idx: idx + self.block_size + 1].long()
        return chunk[:-1], chunk[1:]
