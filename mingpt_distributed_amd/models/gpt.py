"""GPT language model (canonical GPT-2 architecture) over the fused MI355X ops.

API parity with the reference ``GPT`` (``/root/reference/mingpt/model.py:234-356``) and with the
upstream minGPT surface the reference README advertises: ``GPT(config)``,
``forward(idx, targets=None) -> (logits, loss)`` with ``ignore_index=-1``,
``generate(idx, max_new_tokens, temperature, do_sample, top_k)``, ``GPT.get_default_config()``,
``GPT.from_pretrained(model_type)``, ``configure_optimizers(train_config)``.

Architecture is the *intended* one: parameter names
``transformer.{wte,wpe,h.i.{ln_1,attn.{c_attn,c_proj},ln_2,mlp.{c_fc,c_proj}},ln_f}`` and
``lm_head`` (tied to ``wte`` by default, so GPT-2 is 124,439,808 params), causal attention,
tanh-GELU between c_fc and c_proj, one output projection, scaled init on every ``*.c_proj.weight``,
learned position embeddings initialised N(0, 0.02) (fixes D1-D10).

Execution: on a GPU tensor every op runs on the hand-written gfx950 kernels through
``ops.fused`` (bf16 compute, fp32 statistics and accumulation).  On CPU the plain-PyTorch
reference ops run (the CPU plumbing config and the numerics oracle).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import reference as R
from ..utils.config import CfgNode
from ..utils.misc import print_model_size
from .config import GPTConfig, PRESETS


class CausalSelfAttention(nn.Module):
    def __init__(self, config: GPTConfig):
        super().__init__()
        D = config.n_embed
        self.c_attn = nn.Linear(D, 3 * D)
        self.c_proj = nn.Linear(D, D)
        self.n_head = config.n_head
        self.attn_drop = config.attn_drop
        self.resid_drop = config.resid_drop

    def forward(self, x):  # CPU / reference path
        return R.self_attention(x, self.c_attn.weight, self.c_attn.bias, self.c_proj.weight,
                                self.c_proj.bias, self.n_head, self.attn_drop, self.resid_drop,
                                self.training)


class MLP(nn.Module):
    def __init__(self, config: GPTConfig):
        super().__init__()
        D = config.n_embed
        self.c_fc = nn.Linear(D, 4 * D)
        self.c_proj = nn.Linear(4 * D, D)
        self.resid_drop = config.resid_drop

    def forward(self, x):
        return R.mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias,
                     self.resid_drop, self.training)


class Block(nn.Module):
    """Pre-LN transformer block (reference ``model.py:171-189``, D5/D6 fixed)."""

    def __init__(self, config: GPTConfig):
        super().__init__()
        self.ln_1 = nn.LayerNorm(config.n_embed, eps=config.layer_norm_eps)
        self.attn = CausalSelfAttention(config)
        self.ln_2 = nn.LayerNorm(config.n_embed, eps=config.layer_norm_eps)
        self.mlp = MLP(config)
        self.config = config

    def forward(self, x, _links=None):
        """``_links`` (GPU path, set by GPT.forward): (previous block's DropLink, this block's)."""
        if x.is_cuda:
            return self._forward_gpu(x, _links or (None, None))
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))

    def _forward_gpu(self, x, links=(None, None)):
        from ..ops.fused import TransformerBlockFn, _bf16

        B, T, D = x.shape
        c = self.config
        p_attn = c.attn_drop if self.training else 0.0
        p_resid = c.resid_drop if self.training else 0.0
        a, m = self.attn, self.mlp
        ps = [self.ln_1.weight, self.ln_1.bias, a.c_attn.weight, a.c_attn.bias, a.c_proj.weight,
              a.c_proj.bias, self.ln_2.weight, self.ln_2.bias, m.c_fc.weight, m.c_fc.bias,
              m.c_proj.weight, m.c_proj.bias]
        y = TransformerBlockFn.run(x.reshape(B * T, D), *[_bf16(p) for p in ps],
                                     (B, T, c.n_head, p_attn, p_resid, c.layer_norm_eps), links)
        return y.view(B, T, D)


class GPT(nn.Module):
    """GPT Language Model."""

    # GPU training path: run each block's MLP residual-dropout backward inside its consumer's
    # LayerNorm backward (ops/fused.py DropLink).  False = every block runs its own
    # dropout_bias_grad pass (same masks, same gradients; the tests compare the two).
    dropout_handoff = True

    @staticmethod
    def get_default_config() -> CfgNode:
        """Upstream-minGPT style config node (``model_type='gpt'`` with dims None)."""
        C = CfgNode()
        C.model_type = "gpt"
        C.n_layer = None
        C.n_head = None
        C.n_embd = None
        C.vocab_size = None
        C.block_size = None
        C.embd_pdrop = 0.1
        C.resid_pdrop = 0.1
        C.attn_pdrop = 0.1
        return C

    def __init__(self, config, verbose: bool = True):
        super().__init__()
        config = _as_gpt_config(config).resolve()
        self.config = config
        self.block_size = config.block_size
        D = config.n_embed
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(config.vocab_size, D),
            wpe=nn.Embedding(config.block_size, D),
            h=nn.ModuleList([Block(config) for _ in range(config.n_layer)]),
            ln_f=nn.LayerNorm(D, eps=config.layer_norm_eps),
        ))
        self.lm_head = nn.Linear(D, config.vocab_size, bias=False)
        if config.tie_weights:
            self.lm_head.weight = self.transformer.wte.weight
        self.apply(self._init_weights)
        for pn, p in self.named_parameters():
            if pn.endswith("c_proj.weight"):
                nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * config.n_layer))
        if verbose:
            print("number of parameters: %.2fM" % (self.num_params() / 1e6,))
            print_model_size(self)

    # -------------------------------------------------------------------------------- params
    def num_params(self, non_embedding: bool = False) -> int:
        """Parameter count excluding ``lm_head`` (as upstream minGPT reports it)."""
        n = sum(p.numel() for p in self.transformer.parameters())
        if non_embedding:
            n -= self.transformer.wpe.weight.numel()
        return n

    def flops_per_token(self, seq_len: Optional[int] = None) -> float:
        """Training FLOPs per token (fwd + bwd = 3x fwd), matmuls only: 6 * (non-embedding params
        + lm_head) + 6 * L * T * d for causal attention (QK^T and PV, half the square each)."""
        c = self.config
        T = seq_len or c.block_size
        n_mm = sum(p.numel() for n, p in self.transformer.h.named_parameters() if p.dim() == 2)
        n_mm += self.lm_head.weight.numel()
        return 6.0 * n_mm + 6.0 * c.n_layer * T * c.n_embed

    @staticmethod
    def _init_weights(module):
        if isinstance(module, nn.Linear):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if module.bias is not None:
                nn.init.zeros_(module.bias)
        elif isinstance(module, nn.Embedding):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
        elif isinstance(module, nn.LayerNorm):
            nn.init.zeros_(module.bias)
            nn.init.ones_(module.weight)

    # -------------------------------------------------------------------------------- forward
    def forward(self, idx: torch.Tensor, targets: Optional[torch.Tensor] = None):
        B, T = idx.shape
        if T > self.block_size:
            raise ValueError(f"Cannot forward sequence of length {T}, block size is only {self.block_size}")
        if idx.is_cuda:
            return self._forward_gpu(idx, targets)
        tr = self.transformer
        x = R.embedding(idx, tr.wte.weight, tr.wpe.weight, self.config.embed_drop, self.training)
        for block in tr.h:
            x = block(x)
        logits = self.lm_head(tr.ln_f(x))
        loss = None
        if targets is not None:
            loss = R.cross_entropy(logits, targets, ignore_index=-1)
        return logits, loss

    def _forward_gpu(self, idx, targets):
        from ..ops.fused import DropLink, EmbeddingFn, HeadFn, HeadLossFn, _bf16

        tr, c = self.transformer, self.config
        if not getattr(self, "_gpu_checked", False):
            c.check_gpu_support()  # before any launch, not mid-step
            self._gpu_checked = True
        p = c.embed_drop if self.training else 0.0
        x = EmbeddingFn.run(idx, _bf16(tr.wte.weight), _bf16(tr.wpe.weight), p)
        # residual-dropout hand-offs: block l's MLP dropout backward runs inside the LayerNorm
        # backward of its consumer (block l+1's ln_1, or ln_f) -- ops/fused.py DropLink
        link = None
        fuse = self.dropout_handoff and self.training and torch.is_grad_enabled() and c.resid_drop > 0
        for block in tr.h:
            out = DropLink(0.0, 0, _bf16(block.mlp.c_proj.bias)) if fuse else None
            x = block(x, _links=(link, out))
            link = out
        B, T, D = x.shape
        x2 = x.reshape(B * T, D)
        V = self.config.vocab_size
        if targets is not None:
            logits, loss = HeadLossFn.run(x2, _bf16(tr.ln_f.weight), _bf16(tr.ln_f.bias),
                                            _bf16(self.lm_head.weight), targets.reshape(-1).contiguous(),
                                            c.layer_norm_eps, link)
            return logits.view(B, T, -1)[..., :V], loss
        logits = HeadFn.run(x2, _bf16(tr.ln_f.weight), _bf16(tr.ln_f.bias), _bf16(self.lm_head.weight),
                              c.layer_norm_eps, link)
        return logits.view(B, T, -1)[..., :V], None

    # -------------------------------------------------------------------------------- generation
    @torch.no_grad()
    def generate(self, idx, max_new_tokens: int, temperature: float = 1.0, do_sample: bool = False,
                 top_k: Optional[int] = None, use_cache: bool = True):
        """Autoregressive decode (reference ``model.py:322-356``).  With ``use_cache`` the prompt is
        prefilled once and every new token attends to a KV cache (fixes D32: O(steps * T^2))."""
        from .generation import generate

        return generate(self, idx, max_new_tokens, temperature=temperature, do_sample=do_sample,
                        top_k=top_k, use_cache=use_cache)

    # -------------------------------------------------------------------------------- optimizer
    def configure_optimizers(self, train_config):
        """Upstream-minGPT API: AdamW with weight decay on Linear weights only."""
        from ..optim import create_optimizer
        from .config import OptimizerConfig

        oc = OptimizerConfig(learning_rate=train_config.learning_rate,
                             weight_decay=train_config.weight_decay, betas=tuple(train_config.betas))
        return create_optimizer(self, oc)

    # -------------------------------------------------------------------------------- pretrained
    @classmethod
    def from_pretrained(cls, model_type: str, source=None, **overrides):
        """Load OpenAI GPT-2 weights (``gpt2``, ``gpt2-medium``, ``gpt2-large``, ``gpt2-xl``).

        ``source`` may be a HF ``GPT2LMHeadModel``, a state dict in HF naming, or a path/dir
        (safetensors or ``torch.save`` state dict).  With no network the weights must be local.
        """
        from .pretrained import load_gpt2

        return load_gpt2(cls, model_type, source=source, **overrides)


def _as_gpt_config(config) -> GPTConfig:
    if isinstance(config, GPTConfig):
        return config
    if isinstance(config, CfgNode):
        d = dict(config.__dict__)
        mt = d.get("model_type")
        dims = [d.get(k) for k in ("n_layer", "n_head", "n_embd")]
        if mt == "gpt" or mt is None:
            mt = None if any(v is not None for v in dims) else mt
        kw = dict(model_type=mt, n_layer=d.get("n_layer"), n_head=d.get("n_head"), n_embed=d.get("n_embd"),
                  vocab_size=d.get("vocab_size"), block_size=d.get("block_size"),
                  embed_drop=d.get("embd_pdrop", 0.1), resid_drop=d.get("resid_pdrop", 0.1),
                  attn_drop=d.get("attn_pdrop", 0.1))
        for k in ("tie_weights", "layer_norm_eps"):
            if k in d:
                kw[k] = d[k]
        # upstream XOR rule: a named preset must not come with explicit dims
        if mt is not None and mt in PRESETS and any(v is not None for v in dims):
            raise ValueError("give either model_type or (n_layer, n_head, n_embd), not both")
        return GPTConfig(**kw)
    if isinstance(config, dict):
        return GPTConfig(**config)
    raise TypeError(f"unsupported config type {type(config)}")
