"""Model / optimizer configuration.

Field names follow the reference ``GPTConfig`` (``/root/reference/mingpt/model.py:38-51``:
``model_type, n_layer, n_head, n_embed, vocab_size, block_size, embed_drop, resid_drop,
attn_drop``) and the upstream-minGPT names are accepted as aliases (``n_embd``,
``embd_pdrop``, ``resid_pdrop``, ``attn_pdrop``).

Preset resolution fixes the reference's inverted logic (defect D8,
``/root/reference/mingpt/model.py:261-296``): explicit dims win; a ``model_type`` alone
selects a preset; a partial set of dims is an error.  The preset table matches
``model.py:269-294``.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional, Tuple

PRESETS = {
    # GPT-1
    "openai-gpt": dict(n_layer=12, n_head=12, n_embed=768),   # 117M params
    # GPT-2
    "gpt2": dict(n_layer=12, n_head=12, n_embed=768),         # 124M params
    "gpt2-medium": dict(n_layer=24, n_head=16, n_embed=1024),  # 350M params
    "gpt2-large": dict(n_layer=36, n_head=20, n_embed=1280),   # 774M params
    "gpt2-xl": dict(n_layer=48, n_head=25, n_embed=1600),      # 1558M params
    # Gopher
    "gopher-44m": dict(n_layer=8, n_head=16, n_embed=512),
    # tiny models
    "gpt-mini": dict(n_layer=6, n_head=6, n_embed=192),
    "gpt-micro": dict(n_layer=4, n_head=4, n_embed=128),
    "gpt-nano": dict(n_layer=3, n_head=3, n_embed=48),
}

_ALIASES = {"n_embd": "n_embed", "embd_pdrop": "embed_drop", "resid_pdrop": "resid_drop",
            "attn_pdrop": "attn_drop"}


@dataclass
class GPTConfig:
    model_type: Optional[str] = "gpt2"
    n_layer: Optional[int] = None
    n_head: Optional[int] = None
    n_embed: Optional[int] = None
    vocab_size: int = 50257
    block_size: int = 1024
    embed_drop: float = 0.1
    resid_drop: float = 0.1
    attn_drop: float = 0.1
    # Extensions (not in the reference):
    tie_weights: bool = True        # GPT-2 ties lm_head to wte (canonical 124,439,808 params)
    layer_norm_eps: float = 1e-5

    def __init__(self, **kwargs):
        for k, v in list(kwargs.items()):
            if k in _ALIASES:
                kwargs.pop(k)
                kwargs.setdefault(_ALIASES[k], v)
        names = {f.name for f in dataclasses.fields(self)}
        for f in dataclasses.fields(self):
            setattr(self, f.name, f.default)
        for k, v in kwargs.items():
            if k not in names:
                raise TypeError(f"GPTConfig got an unexpected keyword argument {k!r}")
            setattr(self, k, v)

    # upstream attribute names, read-only aliases
    @property
    def n_embd(self):
        return self.n_embed

    @property
    def embd_pdrop(self):
        return self.embed_drop

    @property
    def resid_pdrop(self):
        return self.resid_drop

    @property
    def attn_pdrop(self):
        return self.attn_drop

    def resolve(self) -> "GPTConfig":
        """Fill dims from ``model_type`` if needed; validate.  Returns self."""
        dims = (self.n_layer, self.n_head, self.n_embed)
        given = [d is not None for d in dims]
        if all(given):
            pass  # explicit dims win; model_type is only a label
        elif not any(given):
            if self.model_type not in PRESETS:
                raise ValueError(f"unknown model_type {self.model_type!r}; known: {sorted(PRESETS)}")
            for k, v in PRESETS[self.model_type].items():
                setattr(self, k, v)
        else:
            raise ValueError("give either all of n_layer/n_head/n_embed or none (preset via model_type)")
        if self.n_embed % self.n_head != 0:
            raise ValueError(f"n_embed={self.n_embed} not divisible by n_head={self.n_head}")
        if self.vocab_size is None or self.block_size is None:
            raise ValueError("vocab_size and block_size must be set")
        return self

    @property
    def head_dim(self) -> int:
        return self.n_embed // self.n_head

    # shapes the gfx950 kernels take (checked on the host before the first GPU launch)
    GPU_MAX_HEAD_DIM = 128

    def gpu_unsupported(self) -> Optional[str]:
        """Why the GPU kernels cannot run this config, or None.  Every kernel reads rows in
        16-byte (8 x bf16) vectors; the attention kernels take any head dim that is a multiple of 8
        up to 128 (csrc/include/attn_common.h ``nks_for``; decode: attention.hip)."""
        if self.n_embed is None or self.n_head is None:
            return "config not resolved"
        hd = self.n_embed // self.n_head
        if self.n_embed % 8:
            return f"n_embed={self.n_embed} must be a multiple of 8 on the GPU"
        if hd % 8 or hd > self.GPU_MAX_HEAD_DIM:
            return (f"head dim {hd} (n_embed/n_head) must be a multiple of 8 in [8, "
                    f"{self.GPU_MAX_HEAD_DIM}] on the GPU")
        return None

    def check_gpu_support(self) -> None:
        why = self.gpu_unsupported()
        if why is not None:
            raise ValueError(f"GPTConfig not supported by the GPU kernels: {why}")

    def __repr__(self):
        kv = ", ".join(f"{f.name}={getattr(self, f.name)!r}" for f in dataclasses.fields(self))
        return f"GPTConfig({kv})"

    def __eq__(self, other):
        return isinstance(other, GPTConfig) and all(
            getattr(self, f.name) == getattr(other, f.name) for f in dataclasses.fields(self))


@dataclass
class OptimizerConfig:
    """Reference ``OptimizerConfig`` (``/root/reference/mingpt/model.py:54-59``)."""
    learning_rate: float = 3e-4
    weight_decay: float = 0.1
    betas: Tuple[float, float] = (0.9, 0.95)
    eps: float = 1e-8
