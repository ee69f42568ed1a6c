"""OpenAI GPT-2 checkpoint loader (upstream ``GPT.from_pretrained``, advertised by the reference
README ``/root/reference/README.md:15`` and its ``generate.ipynb``).

Our parameter names are the HuggingFace ``GPT2LMHeadModel`` names, so the mapping is 1:1 except
that HF stores ``c_attn``/``c_proj``/``c_fc`` as ``Conv1D`` weights ``[in, out]``: those four
are transposed into ``nn.Linear`` layout ``[out, in]``.  The ``attn.bias`` / ``attn.masked_bias``
mask buffers are dropped (we have no mask buffers).  Every key and shape is checked.

Sources (no network here): a ``GPT2LMHeadModel`` instance, a state dict with HF names, a
directory / file holding ``model.safetensors`` or a ``torch.save`` state dict (loaded with
``weights_only=True``), or -- if nothing is given -- ``transformers`` with
``local_files_only=True`` (works only when the weights are already in the local HF cache).
"""
from __future__ import annotations

import os
from typing import Dict

import torch

from .config import GPTConfig

_TRANSPOSED = ("attn.c_attn.weight", "attn.c_proj.weight", "mlp.c_fc.weight", "mlp.c_proj.weight")


def _read_state_dict(source) -> Dict[str, torch.Tensor]:
    if isinstance(source, dict):
        return source
    if hasattr(source, "state_dict"):
        return source.state_dict()
    if isinstance(source, str):
        path = source
        if os.path.isdir(path):
            for name in ("model.safetensors", "pytorch_model.bin", "model.pt"):
                if os.path.exists(os.path.join(path, name)):
                    path = os.path.join(path, name)
                    break
        if path.endswith(".safetensors"):
            from safetensors.torch import load_file

            return load_file(path)
        return torch.load(path, map_location="cpu", weights_only=True)
    raise TypeError(f"unsupported checkpoint source {type(source)}")


def hf_to_mingpt(sd_hf: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in sd_hf.items():
        if k.endswith(".attn.masked_bias") or k.endswith(".attn.bias"):
            continue
        if not k.startswith("transformer.") and k != "lm_head.weight":
            k = "transformer." + k  # bare GPT2Model state dicts
        if any(k.endswith(t) for t in _TRANSPOSED):
            v = v.t()
        out[k] = v.contiguous()
    if "lm_head.weight" not in out:
        out["lm_head.weight"] = out["transformer.wte.weight"]
    return out


def load_gpt2(cls, model_type: str, source=None, **overrides):
    assert model_type in {"gpt2", "gpt2-medium", "gpt2-large", "gpt2-xl"}, model_type
    if source is None:
        from transformers import GPT2LMHeadModel

        source = GPT2LMHeadModel.from_pretrained(model_type, local_files_only=True)
    sd_hf = hf_to_mingpt(_read_state_dict(source))
    cfg = GPTConfig(model_type=model_type, vocab_size=50257, block_size=1024, **overrides)
    model = cls(cfg, verbose=False)
    sd = model.state_dict()
    keys = [k for k in sd if not k.endswith(".attn.bias")]
    missing = [k for k in keys if k not in sd_hf]
    extra = [k for k in sd_hf if k not in sd]
    if missing or extra:
        raise KeyError(f"checkpoint mismatch: missing {missing[:5]}..., unexpected {extra[:5]}...")
    with torch.no_grad():
        for k in keys:
            if sd_hf[k].shape != sd[k].shape:
                raise ValueError(f"shape mismatch for {k}: {tuple(sd_hf[k].shape)} vs {tuple(sd[k].shape)}")
            sd[k].copy_(sd_hf[k])
    return model
