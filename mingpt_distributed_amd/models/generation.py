"""Autoregressive generation with a KV cache.

Semantics follow the reference ``GPT.generate`` (``/root/reference/mingpt/model.py:322-356``):
crop the context to ``block_size``, logits of the last position / temperature, optional top-k
masking to -inf, softmax, multinomial sample or greedy top-1, append.  The reference re-runs the
full forward over the prefix for every token (defect D32); here the prompt is prefilled once and
each new token attends to cached keys/values.

GPU path: the prefill runs the gfx950 kernels and keeps each layer's qkv GEMM output as the cache
([B, Tmax, 3D] rows); each decode step runs LN / GEMM / decode-attention kernels on B rows and
appends K/V inside the attention kernel.  CPU path: the same algorithm in plain PyTorch.  When the
sequence outgrows ``block_size`` the window slides and the cache is rebuilt from the cropped
context (exactly the reference's cropping semantics).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from ..ops import reference as R
from ..ops.grads import before_use


def _sample(logits, temperature, do_sample, top_k):
    if not do_sample:  # greedy: top-1 of softmax(logits / t) is the argmax of the logits
        return logits.argmax(dim=-1, keepdim=True)
    logits = logits.float() / temperature
    if top_k is not None:
        v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
        logits[logits < v[:, [-1]]] = -float("Inf")
    probs = F.softmax(logits, dim=-1)
    if do_sample:
        return torch.multinomial(probs, num_samples=1)
    _, idx_next = torch.topk(probs, k=1, dim=-1)
    return idx_next


# ------------------------------------------------------------------------------------ CPU
class _CpuCache:
    def __init__(self, model, idx):
        self.model = model
        self.k, self.v = [], []
        self.logits = self._prefill(idx)

    def _prefill(self, idx):
        m = self.model
        tr = m.transformer
        B, T = idx.shape
        x = tr.wte.weight[idx] + tr.wpe.weight[:T]
        for blk in tr.h:
            h = blk.ln_1(x)
            C = x.shape[-1]
            q, k, v = F.linear(h, blk.attn.c_attn.weight, blk.attn.c_attn.bias).split(C, dim=2)
            H = m.config.n_head
            f = lambda t: t.view(B, T, H, C // H).transpose(1, 2)
            q, k, v = f(q), f(k), f(v)
            self.k.append(k)
            self.v.append(v)
            y = R.causal_attention(q, k, v, 0.0, False).transpose(1, 2).reshape(B, T, C)
            x = x + F.linear(y, blk.attn.c_proj.weight, blk.attn.c_proj.bias)
            x = x + blk.mlp(blk.ln_2(x))
        return m.lm_head(tr.ln_f(x[:, -1]))

    def step(self, tok, pos):
        m = self.model
        tr = m.transformer
        B = tok.shape[0]
        x = tr.wte.weight[tok[:, 0]] + tr.wpe.weight[pos]
        x = x.unsqueeze(1)
        H = m.config.n_head
        for i, blk in enumerate(tr.h):
            h = blk.ln_1(x)
            C = x.shape[-1]
            q, k, v = F.linear(h, blk.attn.c_attn.weight, blk.attn.c_attn.bias).split(C, dim=2)
            f = lambda t: t.view(B, 1, H, C // H).transpose(1, 2)
            q, k, v = f(q), f(k), f(v)
            self.k[i] = torch.cat([self.k[i], k], dim=2)
            self.v[i] = torch.cat([self.v[i], v], dim=2)
            att = (q @ self.k[i].transpose(-1, -2)) / (C // H) ** 0.5
            y = (F.softmax(att, dim=-1) @ self.v[i]).transpose(1, 2).reshape(B, 1, C)
            x = x + F.linear(y, blk.attn.c_proj.weight, blk.attn.c_proj.bias)
            x = x + blk.mlp(blk.ln_2(x))
        return m.lm_head(tr.ln_f(x[:, -1]))


# ------------------------------------------------------------------------------------ GPU
def bf16_weights(model):
    """bf16 view of every weight the decode kernels read, converted ONCE and cached on the model.

    A model trained through the engine already holds bf16 compute weights (returned as is); an
    fp32 model (e.g. ``from_pretrained`` without ``.to(bfloat16)``) gets one bf16 copy per
    weight, reused across decode steps and ``generate`` calls, and refreshed only when the weight
    changes (storage pointer or in-place version).  The captured decode hipGraph therefore holds
    no conversion kernels: per-token traffic is the bf16 weights once."""
    cache = model.__dict__.setdefault("_mg_bf16_weights", {})

    def get(w: torch.Tensor) -> torch.Tensor:
        if w.dtype == torch.bfloat16:
            return w
        stamp = (w.data_ptr(), w._version)
        ent = cache.get(id(w))
        if ent is None or ent[0] != stamp:
            ent = (stamp, w.detach().to(torch.bfloat16).contiguous())
            cache[id(w)] = ent
        return ent[1]

    return get


class _GpuCache:
    """KV caches ([B, Tmax, 3D] qkv rows per layer) plus the captured decode steps of one model at
    one batch size.  Kept on the model across ``generate`` calls (``_gpu_cache``): a later call
    with the same batch re-prefills into the same buffers and replays the same hipGraphs, unless
    a weight changed storage or version since the capture (then the graphs are re-captured)."""

    def __init__(self, model, idx, tmax):
        from ..ops._ext import ext
        from ..ops import gemm as G

        model.config.check_gpu_support()
        self.C, self.G, self.bf = ext(), G, bf16_weights(model)
        self.model = model
        self.tmax = tmax
        B, T = idx.shape
        cfg = model.config
        D = cfg.n_embed
        self.B = B
        self.caches = [torch.empty(B, tmax, 3 * D, device=idx.device, dtype=torch.bfloat16)
                       for _ in range(cfg.n_layer)]
        # decode-attention workspace owned by this state (split partials + per-(b, h) counters
        # that the kernel leaves zero): the captured graphs bake these pointers in
        H = cfg.n_head
        self.dec_part = torch.empty(self.C.attention_decode_part_floats(B, H, D // H),
                                    device=idx.device, dtype=torch.float32)
        self.dec_cnt = torch.zeros(B * H, device=idx.device, dtype=torch.int32)
        self.stamp = _weight_stamp(model)
        self.logits = self._run(idx, 0)

    def prefill(self, idx):
        self.logits = self._run(idx, 0)
        return self.logits

    def _run(self, idx, pos0, pos_dev=None, greedy=None):
        """Prefill (pos0 == 0) or one decode step at position pos0 (or at ``pos_dev[0]``, an int32
        device scalar, when captured in a hipGraph).  ``greedy`` = (tok [B, 1] int64, pos_dev,
        seq [B, Tmax + 1] int64, part [B, G] int64 or None): the step needs nothing from the host.
        With ``part`` (LM head on the skinny GEMM, V > 8192) the LM-head kernel leaves one argmax
        key per (row, workgroup) in part and advances pos_dev, and the NEXT step's embedding
        kernel reduces the keys into its input token (also written to tok and seq[:, pos]) --
        no cross-workgroup hand-off inside a kernel.  Without it the argmax runs in torch and
        writes tok and seq[:, pos + 1] itself."""
        C, G, bf = self.C, self.G, self.bf
        m = self.model
        tr, cfg = m.transformer, m.config
        B, T = idx.shape
        D, H, eps = cfg.n_embed, cfg.n_head, cfg.layer_norm_eps
        wpe = bf(tr.wpe.weight)
        # decode rows (B <= 8) go through the skinny GEMM (gemv.hip): at M = B the MFMA GEMM has
        # one row tile and walks K latency-bound; prefill uses the MFMA GEMM
        skinny = pos0 > 0 and C.gemv_supported(B * T, 4 * D)
        V = cfg.vocab_size
        part = greedy[3] if greedy is not None else None
        if part is not None:  # fused greedy: the token is the argmax of the previous LM head
            x = C.embedding_fwd(idx, bf(tr.wte.weight), wpe, 0.0, 0, pos_dev, part,
                                greedy[2]).view(B * T, D)
        elif pos0 == 0:
            x = C.embedding_fwd(idx.contiguous(), bf(tr.wte.weight), wpe, 0.0, 0).view(B * T, D)
        elif pos_dev is not None:  # the position row is picked on the device (one kernel)
            x = C.embedding_fwd(idx.contiguous(), bf(tr.wte.weight), wpe, 0.0, 0, pos_dev).view(B * T, D)
        else:  # single token at position pos0
            x = C.embedding_fwd(idx.contiguous(), bf(tr.wte.weight), wpe[pos0:pos0 + 1], 0.0, 0).view(B * T, D)

        def lin(inp, w, b, epi, resid=None, ld=0, ln=None, am=None):
            """epi(LN(inp) @ w^T + b) with ``ln`` = a LayerNorm module applied first (fused into
            the skinny GEMM's staging at decode time)."""
            if skinny:
                code = {"none": 0, "bias": 1, "gelu": 2, "resid": 3}[epi]
                lw, lb = (bf(ln.weight), bf(ln.bias)) if ln is not None else (None, None)
                if am is not None:
                    return C.gemv(inp, bf(w), code, None, None, ld, lw, lb, eps, am[0], am[1])
                return C.gemv(inp, bf(w), code, bf(b) if b is not None else None, resid, ld, lw, lb, eps)
            if ln is not None:
                inp, _, _ = C.layernorm_fwd(inp, bf(ln.weight), bf(ln.bias), eps)
            if epi == "gelu":
                pre = torch.empty((inp.shape[0], w.shape[0]), dtype=torch.bfloat16, device=inp.device)
                return G.gemm_nt(inp, bf(w), bias=bf(b), epi="gelu", pre_out=pre)
            return G.gemm_nt(inp, bf(w), bias=bf(b) if b is not None else None, epi=epi, resid=resid,
                             ld=ld or None)

        for i, blk in enumerate(tr.h):
            a, mm = blk.attn, blk.mlp
            qkv = lin(x, a.c_attn.weight, a.c_attn.bias, "bias", ln=blk.ln_1)
            if pos0 == 0:
                self.caches[i][:, :T].copy_(qkv.view(B, T, 3 * D))
                y, _, _ = C.attention_fwd(qkv, B, T, H, 0.0, 0)
            else:
                y = C.attention_decode(qkv, self.caches[i], H, pos0, pos_dev, self.dec_part, self.dec_cnt)
            x = lin(y, a.c_proj.weight, a.c_proj.bias, "resid", resid=x)
            u = lin(x, mm.c_fc.weight, mm.c_fc.bias, "gelu", ln=blk.ln_2)
            x = lin(u, mm.c_proj.weight, mm.c_proj.bias, "resid", resid=x)
        last = x.view(B, T, D)[:, -1].contiguous()
        am = (part, pos_dev) if part is not None else None
        logits = lin(last, m.lm_head.weight, None, "none", ld=(V + 7) // 8 * 8, ln=tr.ln_f, am=am)
        if greedy is not None and part is None:  # small vocab (no fused argmax): same in torch
            tok, pd, seq, _ = greedy
            nxt = logits[:, :V].argmax(-1)
            tok.view(B).copy_(nxt)
            seq.index_copy_(1, (pd.long() + 1), nxt.view(B, 1))
            pd.add_(1)
        return logits[:, :V]

    def _fresh(self):
        st = _weight_stamp(self.model)
        if st != self.stamp:  # a weight moved or changed: captured pointers / bf16 copies are stale
            self.stamp = st
            self.__dict__.pop("_graph", None)
            self.__dict__.pop("_ggraph", None)

    def step(self, tok, pos):
        """One decode step.  Decoding is launch-bound (B rows through ~5 kernels per layer), so
        the step is captured once as a hipGraph over static token / position buffers and
        replayed; the KV caches are persistent buffers the captured kernels append to."""
        if not _GRAPH_DECODE:
            return self._run(tok, pos)
        self._fresh()
        g = getattr(self, "_graph", None)
        if g is None:
            g = self._graph = {"tok": tok.clone(), "pos": torch.full((1,), pos, dtype=torch.int32,
                                                                     device=tok.device)}
            self._run(g["tok"], pos, g["pos"])  # warm-up (workspaces, lazy kernel attributes)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                g["logits"] = self._run(g["tok"], max(pos, 1), g["pos"])
            g["graph"] = graph
        g["tok"].copy_(tok)
        g["pos"].fill_(pos)
        g["graph"].replay()
        return g["logits"]

    def greedy(self, tok, pos, n):
        """n greedy decode steps starting with token ``tok`` [B, 1] at position ``pos``: the captured
        step takes its input token and position from device buffers that its own kernels advance
        (fused argmax, see ``_run``), so the n replays are queued back to back without a host round
        trip.  Returns the n new tokens [B, n] (positions pos + 1 .. pos + n)."""
        assert pos + n <= self.tmax
        B = tok.shape[0]
        self._fresh()
        g = getattr(self, "_ggraph", None)
        cfg = self.model.config
        fused = self.C.gemv_supported(B, 4 * cfg.n_embed) and cfg.vocab_size > 8192
        if g is None:
            dev = tok.device
            g = {"tok": tok.clone(), "pos": torch.full((1,), pos, dtype=torch.int32, device=dev),
                 "seq": torch.zeros(B, self.tmax + 1, dtype=torch.long, device=dev),
                 "part": (torch.zeros(B, self.C.gemv_argmax_groups(cfg.vocab_size, B), dtype=torch.long,
                                      device=dev) if fused else None)}
            self._ggraph = g  # workspaces are allocated outside the capture (eager warm-up step)
            self._greedy_seed(g, tok, pos)
            self._run(g["tok"], max(pos, 1), g["pos"], (g["tok"], g["pos"], g["seq"], g["part"]))
        if _GRAPH_DECODE and "graph" not in g:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                self._run(g["tok"], max(pos, 1), g["pos"], (g["tok"], g["pos"], g["seq"], g["part"]))
            g["graph"] = graph
        self._greedy_seed(g, tok, pos)
        for _ in range(n):
            if _GRAPH_DECODE:
                g["graph"].replay()
            else:
                self._run(g["tok"], max(pos, 1), g["pos"], (g["tok"], g["pos"], g["seq"], g["part"]))
        if g["part"] is None:
            return g["seq"][:, pos + 1:pos + 1 + n]
        # the last step's token is still in its LM-head keys: reduce them here (unsigned max =
        # signed max after flipping the top bit; low word = 0xffffffff - column)
        k = (g["part"] ^ _I64_MIN).max(dim=1).values ^ _I64_MIN
        last = 0xFFFFFFFF - (k & 0xFFFFFFFF)
        return torch.cat([g["seq"][:, pos + 1:pos + n], last.view(B, 1)], dim=1)

    @staticmethod
    def _greedy_seed(g, tok, pos):
        """Point the greedy loop's device state at token ``tok`` [B, 1] at position ``pos``."""
        g["tok"].copy_(tok)
        g["pos"].fill_(pos)
        if g["part"] is not None:  # keys that every real logit loses to, argmax = tok
            g["part"].zero_()
            g["part"][:, :1].copy_(-1 - tok)  # bits 0xffffffff_(0xffffffff - tok)


_I64_MIN = -(1 << 63)


def _weight_stamp(model):
    return tuple((p.data_ptr(), p._version) for p in model.parameters())


def _gpu_cache(model, idx, tmax):
    """The model's decode state for this batch size (re-prefilled), or a new one."""
    c = model.__dict__.get("_mg_decode_cache")
    if c is not None and c.B == idx.size(0) and c.tmax == tmax and c.caches[0].device == idx.device:
        c.prefill(idx)
        return c
    c = _GpuCache(model, idx, tmax)
    model.__dict__["_mg_decode_cache"] = c
    return c


_GRAPH_DECODE = True  # set False to launch the decode step eagerly


@torch.no_grad()
def generate(model, idx, max_new_tokens: int, temperature: float = 1.0, do_sample: bool = False,
             top_k: Optional[int] = None, use_cache: bool = True):
    bs = model.block_size
    # ZeRO-1: the KV-cache path launches the kernels directly (never model.forward), so neither
    # the fused ops' per-bucket waits nor the engine's forward pre-hook run: wait here for every
    # in-flight parameter all-gather (stream-ordered) before any decode kernel reads the weights
    before_use(*model.parameters())
    if not use_cache:
        for _ in range(max_new_tokens):
            idx_cond = idx if idx.size(1) <= bs else idx[:, -bs:]
            logits, _ = model(idx_cond)
            idx = torch.cat((idx, _sample(logits[:, -1, :], temperature, do_sample, top_k)), dim=1)
        return idx
    if idx.is_cuda and not do_sample and max_new_tokens > 0:
        return _generate_greedy_gpu(model, idx, max_new_tokens)
    cache = None
    for _ in range(max_new_tokens):
        T = idx.size(1)
        if cache is None or T > bs:
            idx_cond = idx if T <= bs else idx[:, -bs:]
            cache = _gpu_cache(model, idx_cond, bs) if idx.is_cuda else _CpuCache(model, idx_cond)
            cache.pos = idx_cond.size(1)
            logits = cache.logits
        idx_next = _sample(logits, temperature, do_sample, top_k)
        idx = torch.cat((idx, idx_next), dim=1)
        if idx.size(1) > bs:
            cache = None  # window slides: rebuild from the cropped context next step
            continue
        logits = cache.step(idx_next, cache.pos)
        cache.pos += 1
    return idx


def _generate_greedy_gpu(model, idx, max_new_tokens):
    """Greedy decode on the GPU: one prefill per context window, then the device-side token loop
    (``_GpuCache.greedy``) for every position the window still has room for.  Once the sequence
    outgrows block_size, each token is a fresh prefill of the last block_size tokens -- the
    reference's crop-every-step semantics (``/root/reference/mingpt/model.py:333``)."""
    bs = model.block_size
    B, T0 = idx.shape
    out = torch.empty(B, T0 + max_new_tokens, dtype=torch.long, device=idx.device)
    out[:, :T0] = idx
    T, end = T0, T0 + max_new_tokens
    while T < end:
        ctx = out[:, max(0, T - bs):T]
        L = ctx.size(1)
        cache = _gpu_cache(model, ctx, bs)
        out[:, T] = cache.logits.argmax(-1)
        T += 1
        n = min(end - T, bs - L)
        if n > 0:
            out[:, T:T + n] = cache.greedy(out[:, T - 1:T], L, n)
            T += n
    return out
