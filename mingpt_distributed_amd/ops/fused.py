"""GPU execution path: autograd Functions over the gfx950 kernels.

Granularity is chosen for the MI355X, not for module boundaries: one Function per transformer
block (LN1 -> QKV GEMM+bias -> flash attention -> proj GEMM with fused bias+dropout+residual ->
LN2 -> FC GEMM with fused bias+GELU -> proj GEMM with fused bias+dropout+residual), one for the
embedding and one for final-LN + LM head + cross-entropy.  Every norm, attention, loss and
elementwise op and every GEMM -- the fused-epilogue ones (bias+GELU, bias+dropout+residual,
GELU', the weight gradients with their fp32 accumulation), the plain ones of a block (qkv
projection, the three data gradients) and the LM head's forward, weight and data gradients -- is
a hand-written HIP kernel (``gemm.hip`` through :mod:`.gemm`): there is one backend, no library
GEMM and no runtime switch to one (hipBLASLt comparisons live in ``bench/`` microbenchmarks only:
``bench/gemm_blas_shapes.py``, ``bench/bench_wgrad_blas.py``).  Weight gradients are accumulated
in fp32 straight into ``param.main_grad`` (see ``grads.py``) so the data-parallel engine can
all-reduce a bucket the moment its last gradient lands.

Reference anchors: block structure ``/root/reference/mingpt/model.py:171-189`` (with D4/D5/D6
fixed), embedding ``model.py:193-231``, head + loss ``model.py:309-320``.
"""
from __future__ import annotations

import torch

from . import gemm as G
from . import streams
from ._ext import ext
from .grads import before_use, finish, grad_target, note_use


class DropLink:
    """Hand-off of one residual-dropout backward between neighbouring fused ops.

    Block l's MLP branch ends in ``x2 = x1 + dropout(c_proj(...))`` (/root/reference/mingpt/model.py:
    188).  Its backward starts with dz = dropout'(dx2) plus the c_proj bias gradient, and dx2 is
    the output of the LayerNorm backward of whatever consumed x2 (block l+1's ln_1 or the final
    ln_f).  That consumer computes dz inside its LayerNorm-backward kernel (layernorm.hip DROP: one
    read of the gradient instead of two) and leaves it here; block l's backward takes it instead of
    running the separate dropout_bias_grad pass.  Created per forward by the producing block; a
    consumer that never ran its backward leaves ``dz`` None and the producer falls back."""

    __slots__ = ("p", "seed", "bias", "dz", "target")

    def __init__(self, p: float, seed: int, bias: torch.Tensor):
        self.p, self.seed, self.bias = p, seed, bias
        self.dz = None
        self.target = None

    def ln_backward(self, C, dh, x, w, mean, rstd, dw, db, dres):
        """The consumer's LayerNorm backward, with this link's dropout backward fused when it
        applies: returns dx and leaves dz + the bias-gradient target for the producer."""
        if self.p <= 0:
            return C.layernorm_bwd(dh, x, w, mean, rstd, dw, db, dres)
        self.target = grad_target(self.bias)
        dx, self.dz = C.layernorm_bwd_dropout(dh, x, w, mean, rstd, dw, db, dres, self.target[0],
                                              float(self.p), int(self.seed))
        return dx


def _ln_backward(C, link, dh, x, w, mean, rstd, dw, db, dres):
    if link is None:
        return C.layernorm_bwd(dh, x, w, mean, rstd, dw, db, dres)
    return link.ln_backward(C, dh, x, w, mean, rstd, dw, db, dres)


def new_seed() -> int:
    """Dropout seed from torch's CPU generator (reproducible under torch.manual_seed, no GPU sync)."""
    return int(torch.randint(1, 2 ** 62, (1,)).item())


def _bf16(t: torch.Tensor) -> torch.Tensor:
    return t if t.dtype == torch.bfloat16 else t.to(torch.bfloat16)


# ------------------------------------------------------------------------------------ embedding

# Decided (measured) fusions, no runtime switches: the MLP fc bias gradient is summed inside the fc2
# data-gradient GEMM's staged epilogue (one add per stored element, one atomic per tile column; no
# separate 400 MB column-sum pass over dpre), and the qkv bias gradient inside the attention backward
# (dK / dV columns per key block in registers, dQ columns by one column-sum pass after the finalize).
# The attention backward's delta = rowsum(dO * O) has its own pass (attn_bwd_pre_kernel): computing
# it in the dO GEMM's epilogue cost the K = 768 projection more than the pass (round 2,
# profiles/round2_s10_delta_epilogue_ab.txt).


def _dgrad(dy, w):
    """dX = dY @ W for a plain (epilogue-free) data gradient (gemm.hip, weight read in place)."""
    return G.gemm_dgrad(dy, w)


def _wgrad(dy, x, target):
    """main_grad += dY^T @ X (gemm.hip split-K, fp32 accumulate in the epilogue).  ``target`` is
    grad_target()'s (buffer, is_main): a main_grad accumulation runs on the weight-gradient
    stream (streams.py), beside the data gradients; a gradient returned to autograd in order."""
    buf, is_main = target
    if is_main:
        streams.run_wgrad(lambda: G.gemm_tn_acc(dy, x, buf), dy, x)
    else:
        G.gemm_tn_acc(dy, x, buf)


class _EngineFn(torch.autograd.Function):
    """Autograd Function over engine-managed parameters.  Call :meth:`run`, not ``apply``: the
    gradient-readiness protocol counts a parameter use only when the CALLER runs with grad
    enabled, and inside ``forward`` autograd has always switched grad mode off (a use counted
    there under ``no_grad`` would never be matched by a backward; one skipped there would let a
    bucket holding a tied weight launch before its second gradient lands)."""

    @classmethod
    def run(cls, *args):
        if torch.is_grad_enabled():
            for a in args:
                if isinstance(a, torch.Tensor) and a.requires_grad:
                    note_use(a)
        return cls.apply(*args)


class EmbeddingFn(_EngineFn):
    @staticmethod
    def forward(ctx, idx, wte, wpe, p):
        before_use(wte, wpe)
        seed = new_seed() if p > 0 else 0
        out = ext().embedding_fwd(idx.contiguous(), wte, wpe, float(p), seed)
        ctx.save_for_backward(idx)
        ctx.params = (wte, wpe)
        ctx.p, ctx.seed = p, seed
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        wte, wpe = ctx.params
        bte, mte = grad_target(wte)
        bpe, mpe = grad_target(wpe)
        ext().embedding_bwd(idx, g.contiguous(), bte, bpe, ctx.p, ctx.seed)
        return None, finish(wte, bte, mte), finish(wpe, bpe, mpe), None


# ------------------------------------------------------------------------------------ block
class TransformerBlockFn(_EngineFn):
    """x [M, D] -> x + attn(ln1(x)) -> (+ mlp(ln2(.)))  with every op on a HIP kernel."""

    @staticmethod
    def forward(ctx, x, ln1w, ln1b, wqkv, bqkv, wo, bo, ln2w, ln2b, wfc, bfc, wp, bp, cfg, links=(None, None)):
        """``links`` = (link_in, link_out): the previous block's MLP-dropout hand-off (computed by
        this block's ln_1 backward) and this block's own (filled by the next consumer)."""
        B, T, H, p_attn, p_resid, eps = cfg
        C = ext()
        before_use(ln1w, ln1b, wqkv, bqkv, wo, bo, ln2w, ln2b, wfc, bfc, wp, bp)
        seeds = (new_seed() if p_attn > 0 else 0, new_seed() if p_resid > 0 else 0,
                 new_seed() if p_resid > 0 else 0)
        h, mean1, rstd1 = C.layernorm_fwd(x, ln1w, ln1b, eps)
        qkv = G.gemm_nt(h, wqkv, bias=bqkv, epi="bias")
        y, lse, amask = C.attention_fwd(qkv, B, T, H, float(p_attn), seeds[0])
        x1 = G.gemm_nt(y, wo, bias=bo, epi="resid", resid=x, p=p_resid, seed=seeds[1])
        h2, mean2, rstd2 = C.layernorm_fwd(x1, ln2w, ln2b, eps)
        # GELU'(z) for the fc2 data gradient: in the fragment order of the W4 tiles when both GEMMs
        # run on them (no LDS staging for that plane in either epilogue), else row-major
        M, N4 = x.shape[0], wfc.shape[0]
        frag = G.frag_aux_ok(M, N4, x.shape[1])
        gd = torch.empty(G.frag_aux_elems(M, N4) if frag else (M, N4), dtype=torch.bfloat16, device=x.device)
        u = G.gemm_nt(h2, wfc, bias=bfc, epi="gelu", pre_out=gd, frag=frag)
        x2 = G.gemm_nt(u, wp, bias=bp, epi="resid", resid=x1, p=p_resid, seed=seeds[2])
        ctx.save_for_backward(x, h, mean1, rstd1, qkv, y, lse, amask, x1, h2, mean2, rstd2, gd, u)
        ctx.params = (ln1w, ln1b, wqkv, bqkv, wo, bo, ln2w, ln2b, wfc, bfc, wp, bp)
        ctx.cfg, ctx.seeds, ctx.frag = cfg, seeds, frag
        link_in, link_out = links
        if link_out is not None:  # the MLP dropout this block's consumer will differentiate
            link_out.p, link_out.seed, link_out.dz = p_resid, seeds[2], None
        ctx.links = links
        return x2

    @staticmethod
    def backward(ctx, dx2):
        B, T, H, p_attn, p_resid, eps = ctx.cfg
        C = ext()
        x, h, mean1, rstd1, qkv, y, lse, amask, x1, h2, mean2, rstd2, gd, u = ctx.saved_tensors
        ln1w, ln1b, wqkv, bqkv, wo, bo, ln2w, ln2b, wfc, bfc, wp, bp = ctx.params
        dx2 = dx2.contiguous()
        g = {}
        for prm in ctx.params:
            g[id(prm)] = grad_target(prm)
        link_in, link_out = ctx.links
        # ---- MLP: x2 = x1 + drop(gelu(h2 Wfc^T + bfc) Wp^T + bp)
        if link_out is not None and link_out.dz is not None:
            # dz = dropout'(dx2) and d(bias) came with dx2 (the consumer's LayerNorm backward)
            dz, g[id(bp)] = link_out.dz, link_out.target
            link_out.dz = link_out.target = None
        elif p_resid > 0:  # dz = dropout'(dx2) and d(bias) in one pass
            dz = C.dropout_bias_grad(dx2, g[id(bp)][0], p_resid, ctx.seeds[2])
        else:
            dz = dx2
            C.bias_grad(dz, g[id(bp)][0])
        _wgrad(dz, u, g[id(wp)])
        # fc bias gradient: column sums of dpre in the GELU' epilogue
        dpre = G.gemm_dgrad(dz, wp, epi="gelu_bwd", aux=gd, dbias=g[id(bfc)][0], aux_frag=ctx.frag)
        _wgrad(dpre, h2, g[id(wfc)])
        dh2 = _dgrad(dpre, wfc)
        # ---- attention: x1 = x + drop(attn(h Wqkv^T + bqkv) Wo^T + bo); the attention branch's
        # dropout backward (dz) and bias gradient come out of ln_2's backward kernel
        if p_resid > 0:
            dx1, dz = C.layernorm_bwd_dropout(dh2, x1, ln2w, mean2, rstd2, g[id(ln2w)][0], g[id(ln2b)][0], dx2,
                                              g[id(bo)][0], float(p_resid), int(ctx.seeds[1]))
        else:
            dx1 = C.layernorm_bwd(dh2, x1, ln2w, mean2, rstd2, g[id(ln2w)][0], g[id(ln2b)][0], dx2)
            dz = dx1
            C.bias_grad(dz, g[id(bo)][0])
        _wgrad(dz, y, g[id(wo)])
        dy = _dgrad(dz, wo)
        # qkv bias gradient summed inside the attention backward
        dqkv = C.attention_bwd(qkv, y, dy, lse, amask, B, T, H, float(p_attn), ctx.seeds[0],
                               g[id(bqkv)][0])
        _wgrad(dqkv, h, g[id(wqkv)])
        dh = _dgrad(dqkv, wqkv)
        dx = _ln_backward(C, link_in, dh, x, ln1w, mean1, rstd1, g[id(ln1w)][0], g[id(ln1b)][0], dx1)
        outs = [finish(prm, *g[id(prm)]) for prm in ctx.params]
        return (dx, *outs, None, None)


# ------------------------------------------------------------------------------------ head + loss
# The LM head's forward ([M, 768] x [768, 50304], K = 768, 13 GB of logits at B = 128), data
# gradient ([M, 50304] x [50304, 768]: the 128x96-wave W4 tile) and weight gradient (fp32
# accumulate into main_grad) all run on gemm.hip.  Training cross-entropy in one pass over the
# logits (xent.hip xent_fused: loss and dlogits = (softmax - onehot) / n_valid written in forward,
# grad_out applied in backward); without gradients (evaluation) the loss-only xent_fwd pass.


class HeadLossFn(_EngineFn):
    """loss = CE(LN_f(x) @ W^T, targets) with padded-vocab logits; returns (logits[M, Vpad], loss)."""

    @staticmethod
    def forward(ctx, x, lnw, lnb, w, targets, eps, link=None):
        C = ext()
        before_use(lnw, lnb, w)
        ctx.link = link  # the last block's MLP-dropout hand-off (DropLink), or None
        V = w.shape[0]
        ld = (V + 127) // 128 * 128
        h, mean, rstd = C.layernorm_fwd(x, lnw, lnb, eps)
        logits = G.gemm_nt(h, w, ld=ld)
        fused = C.xent_fused(logits, targets, V) if any(ctx.needs_input_grad) else []
        if fused:  # the backward never reads the logits again
            out, dlogits = fused
            ctx.save_for_backward(x, h, mean, rstd, dlogits, None, None, out)
        else:
            out, lse = C.xent_fwd(logits, targets, V)
            ctx.save_for_backward(x, h, mean, rstd, logits, targets, lse, out)
        ctx.fused = bool(fused)
        ctx.params = (lnw, lnb, w)
        ctx.eps = eps
        ctx.mark_non_differentiable(logits)
        ctx.set_materialize_grads(False)  # never build a [M, Vpad] zero grad for the logits
        return logits, out[0]

    @staticmethod
    def backward(ctx, _dlogits, dloss):
        C = ext()
        x, h, mean, rstd, logits, targets, lse, out = ctx.saved_tensors
        lnw, lnb, w = ctx.params
        V = w.shape[0]
        gscale = dloss.reshape(1).float().contiguous()
        if ctx.fused:
            dlogits = logits
            C.xent_scale_(dlogits, gscale)  # no-op on the device when grad_out == 1
        else:
            dlogits = C.xent_bwd(logits, targets, lse, gscale, out, V)
        del logits
        bw, mw = grad_target(w)
        G.gemm_tn_acc(dlogits, h, bw, n_valid=V)
        dh = G.gemm_dgrad(dlogits, w)  # W^T padded to the logits' row stride (zero columns)
        blw, mlw = grad_target(lnw)
        blb, mlb = grad_target(lnb)
        dx = _ln_backward(C, ctx.link, dh, x, lnw, mean, rstd, blw, blb, None)
        return dx, finish(lnw, blw, mlw), finish(lnb, blb, mlb), finish(w, bw, mw), None, None, None


class HeadFn(_EngineFn):
    """logits = LN_f(x) @ W^T (inference / custom-loss path). Gradient flows to x and weights."""

    @staticmethod
    def forward(ctx, x, lnw, lnb, w, eps, link=None):
        C = ext()
        before_use(lnw, lnb, w)
        ctx.link = link
        V = w.shape[0]
        ld = (V + 7) // 8 * 8
        h, mean, rstd = C.layernorm_fwd(x, lnw, lnb, eps)
        logits = G.gemm_nt(h, w, ld=ld)
        ctx.save_for_backward(x, h, mean, rstd)
        ctx.params = (lnw, lnb, w)
        ctx.eps, ctx.ld = eps, ld
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        C = ext()
        x, h, mean, rstd = ctx.saved_tensors
        lnw, lnb, w = ctx.params
        V = w.shape[0]
        dl = dlogits.contiguous().to(torch.bfloat16)
        if ctx.ld > V:
            dl[:, V:] = 0
        bw, mw = grad_target(w)
        G.gemm_tn_acc(dl, h, bw, n_valid=V)
        dh = G.gemm_nn(dl, w)
        blw, mlw = grad_target(lnw)
        blb, mlb = grad_target(lnb)
        dx = _ln_backward(C, ctx.link, dh, x, lnw, mean, rstd, blw, blb, None)
        return dx, finish(lnw, blw, mlw), finish(lnb, blb, mlb), finish(w, bw, mw), None, None
