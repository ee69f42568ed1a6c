"""GPT-2 byte-level BPE tokenizer (the ``mingpt/bpe.py`` capability advertised by the reference
README, ``/root/reference/README.md:10``).

* :func:`bytes_to_unicode` -- the reversible byte <-> printable-unicode table GPT-2 uses so that
  every byte sequence is a string of "visible" characters.
* :class:`Encoder` -- ``encode(text) -> ids`` / ``decode(ids) -> text`` given the
  ``encoder.json`` token->id map and the ``vocab.bpe`` merge list; pre-tokenises with the GPT-2
  regex and applies merges by rank with a per-word cache.
* :class:`BPETokenizer` -- ``tok(text) -> LongTensor[1, T]`` and ``tok.decode(tensor)``.

No network is assumed: :func:`get_encoder` looks for ``encoder.json`` / ``vocab.bpe`` in
``$MINGPT_BPE_DIR`` or ``~/.cache/mingpt`` and raises a clear error if they are missing.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, List, Sequence, Tuple

import regex as re
import torch

GPT2_PATTERN = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""


def bytes_to_unicode() -> Dict[int, str]:
    """Map every byte 0..255 to a unicode char; printable bytes map to themselves."""
    keep = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    table = {b: chr(b) for b in keep}
    extra = 0
    for b in range(256):
        if b not in table:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def get_pairs(word: Sequence[str]) -> set:
    return {(word[i], word[i + 1]) for i in range(len(word) - 1)}


class Encoder:
    def __init__(self, encoder: Dict[str, int], bpe_merges: Iterable[Tuple[str, str]]):
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        self.encoder = dict(encoder)
        self.decoder = {v: k for k, v in self.encoder.items()}
        self.bpe_ranks = {tuple(m): i for i, m in enumerate(bpe_merges)}
        self.pat = re.compile(GPT2_PATTERN)
        self.cache: Dict[str, str] = {}

    def bpe(self, token: str) -> str:
        """Merge the characters of one pre-token by merge rank; returns space-joined parts."""
        if token in self.cache:
            return self.cache[token]
        word = list(token)
        while len(word) > 1:
            pairs = get_pairs(word)
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            first, second = best
            merged: List[str] = []
            i = 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == first and word[i + 1] == second:
                    merged.append(first + second)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = merged
        out = " ".join(word)
        self.cache[token] = out
        return out

    def encode(self, text: str) -> List[int]:
        ids: List[int] = []
        for tok in self.pat.findall(text):
            tok_u = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[p] for p in self.bpe(tok_u).split(" "))
        return ids

    def decode(self, ids: Iterable[int]) -> str:
        s = "".join(self.decoder[int(i)] for i in ids)
        return bytes(self.byte_decoder[c] for c in s).decode("utf-8", errors="replace")


def _bpe_dir() -> str:
    return os.environ.get("MINGPT_BPE_DIR", os.path.join(os.path.expanduser("~"), ".cache", "mingpt"))


def load_merges(path: str) -> List[Tuple[str, str]]:
    with open(path, "r", encoding="utf-8") as f:
        lines = f.read().split("\n")
    out = []
    for line in lines[1:]:  # first line is a version header
        if line.strip():
            a, b = line.split()
            out.append((a, b))
    return out


def get_encoder(directory: str = None) -> Encoder:
    d = directory or _bpe_dir()
    enc_p, bpe_p = os.path.join(d, "encoder.json"), os.path.join(d, "vocab.bpe")
    if not (os.path.exists(enc_p) and os.path.exists(bpe_p)):
        raise FileNotFoundError(
            f"GPT-2 BPE files not found in {d} (need encoder.json and vocab.bpe). There is no network "
            "access here: place the OpenAI files there or set MINGPT_BPE_DIR.")
    with open(enc_p, "r", encoding="utf-8") as f:
        encoder = json.load(f)
    return Encoder(encoder, load_merges(bpe_p))


class BPETokenizer:
    """Callable tokenizer: ``tok("text") -> LongTensor[1, T]``; ``tok.decode(ids) -> str``."""

    def __init__(self, encoder: Encoder = None, directory: str = None):
        self.encoder = encoder if encoder is not None else get_encoder(directory)

    def __call__(self, text: str, return_tensors: str = "pt") -> torch.Tensor:
        assert return_tensors == "pt"
        assert isinstance(text, str)
        return torch.tensor([self.encoder.encode(text)], dtype=torch.long)

    def decode(self, idx: torch.Tensor) -> str:
        assert idx.ndim == 1
        return self.encoder.decode(idx.tolist())
