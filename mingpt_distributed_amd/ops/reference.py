"""Plain-PyTorch implementations of every fused op.

These serve two roles only: the CPU execution path (BASELINE config #1, gpt-nano on
SortDataset, and the multi-process ``gloo`` tests) and the fp32 numerics oracle that the
HIP kernels are tested against.  On a GPU tensor the framework never calls these (see
``ops/__init__.py``): the HIP kernels in ``csrc/kernels`` run instead.

Semantics are the *intended* ones of the reference (``/root/reference/mingpt/model.py``):
causal attention with a -inf mask (fixes D4), GELU between c_fc and c_proj (fixes D5),
tanh-approximate GELU (upstream ``NewGELU``, so OpenAI GPT-2 weights reproduce), and
cross-entropy with ``ignore_index=-1`` (``model.py:316-318``).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

GELU_K0 = math.sqrt(2.0 / math.pi)
GELU_K1 = 0.044715


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * x * (1.0 + torch.tanh(GELU_K0 * (x + GELU_K1 * x * x * x)))


def embedding(idx, wte, wpe, p: float, training: bool):
    B, T = idx.shape
    x = wte[idx] + wpe[:T].unsqueeze(0)
    return F.dropout(x, p, training)


def layer_norm(x, w, b, eps: float = 1e-5):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def linear(x, w, b=None):
    return F.linear(x, w, b)


def causal_attention(q, k, v, p: float, training: bool):
    """q, k, v: [B, H, T, hd] -> [B, H, T, hd]. Explicit masked softmax (upstream minGPT)."""
    T = q.size(-2)
    att = (q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(k.size(-1)))
    mask = torch.ones(T, T, dtype=torch.bool, device=q.device).tril()
    att = att.masked_fill(~mask, float("-inf"))
    att = F.softmax(att, dim=-1)
    att = F.dropout(att, p, training)
    return att @ v


def self_attention(x, w_attn, b_attn, w_proj, b_proj, n_head: int, attn_p: float, resid_p: float,
                   training: bool):
    B, T, C = x.shape
    q, k, v = linear(x, w_attn, b_attn).split(C, dim=2)
    q = q.view(B, T, n_head, C // n_head).transpose(1, 2)
    k = k.view(B, T, n_head, C // n_head).transpose(1, 2)
    v = v.view(B, T, n_head, C // n_head).transpose(1, 2)
    y = causal_attention(q, k, v, attn_p, training)
    y = y.transpose(1, 2).contiguous().view(B, T, C)
    return F.dropout(linear(y, w_proj, b_proj), resid_p, training)


def mlp(x, w_fc, b_fc, w_proj, b_proj, resid_p: float, training: bool):
    return F.dropout(linear(gelu_tanh(linear(x, w_fc, b_fc)), w_proj, b_proj), resid_p, training)


def cross_entropy(logits, targets, ignore_index: int = -1):
    return F.cross_entropy(logits.reshape(-1, logits.size(-1)).float(), targets.reshape(-1),
                           ignore_index=ignore_index)
