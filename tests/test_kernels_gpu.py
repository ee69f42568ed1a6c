"""Numerics of the standalone gfx950 kernels vs plain-PyTorch fp32 references.

Each kernel is called through the raw extension (``_C``) so a failure points at one kernel.
"""
import math

import pytest
import torch

from mingpt_distributed_amd.ops import reference as R
from mingpt_distributed_amd.ops._ext import ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV, torch.bfloat16)


def _close(a, b, atol, rtol=0.02):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=rtol)


@pytest.mark.parametrize("M,D", [(64, 48), (1000, 768), (257, 1600), (33, 192)])
def test_layernorm_fwd_bwd(M, D):
    C = ext()
    x, w, b = _bf(M, D, seed=1), _bf(D, seed=2) * 0.1 + 1, _bf(D, seed=3) * 0.1
    y, mean, rstd = C.layernorm_fwd(x, w, b, 1e-5)
    xr, wr, br = (t.float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
    _close(y, yr, atol=3e-2)
    torch.testing.assert_close(mean, xr.mean(-1).detach(), atol=1e-3, rtol=1e-3)
    dy = _bf(M, D, seed=4)
    yr.backward(dy.float())
    dw = torch.zeros(D, device=DEV)
    db = torch.ones(D, device=DEV)  # accumulates into existing main grad
    dx = C.layernorm_bwd(dy, x, w, mean, rstd, dw, db, None)
    _close(dx, xr.grad, atol=5e-2)
    res = _bf(M, D, seed=5)
    dx2 = C.layernorm_bwd(dy, x, w, mean, rstd, torch.zeros_like(dw), torch.zeros_like(db), res)
    _close(dx2, xr.grad + res.float(), atol=6e-2)
    torch.testing.assert_close(dw, wr.grad, atol=5e-2 * math.sqrt(M) / 4, rtol=2e-2)
    torch.testing.assert_close(db - 1, br.grad, atol=5e-2 * math.sqrt(M) / 4, rtol=2e-2)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_embedding(p):
    C = ext()
    B, T, V, D = 4, 64, 97, 192
    idx = torch.randint(0, V, (B, T), device=DEV)
    wte, wpe = _bf(V, D, seed=5), _bf(T * 2, D, seed=6)
    out = C.embedding_fwd(idx, wte, wpe, p, 1234)
    ref = wte.float()[idx] + wpe.float()[:T].unsqueeze(0)
    scale = 65536.0 / (65536 - round(65536 * p))  # the 16-bit keep scale (common.h rowdrop)
    if p == 0.0:
        _close(out, ref, atol=2e-2)
    else:
        keep = out.float() != 0
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p)) < 0.02
        _close(out.float()[keep], (ref * scale)[keep], atol=3e-2)
    dout = _bf(B, T, D, seed=7)
    dwte = torch.zeros(V, D, device=DEV)
    dwpe = torch.zeros(T * 2, D, device=DEV)
    C.embedding_bwd(idx, dout, dwte, dwpe, p, 1234)
    g = dout.float()
    if p > 0:  # the mask from a forward over an all-ones table (a real output can be exactly 0)
        ones = C.embedding_fwd(idx, torch.ones_like(wte), torch.zeros_like(wpe), p, 1234)
        g = g * (ones.float() != 0).float() * scale
    ref_wte = torch.zeros(V, D, device=DEV).index_add_(0, idx.flatten(), g.reshape(-1, D))
    ref_wpe = torch.zeros(T * 2, D, device=DEV)
    ref_wpe[:T] = g.sum(0)
    torch.testing.assert_close(dwte, ref_wte, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(dwpe, ref_wpe, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("M,V,ld", [(64, 65, 72), (300, 50257, 50304), (17, 3, 8)])
def test_cross_entropy(M, V, ld):
    C = ext()
    logits = _bf(M, ld, scale=3.0, seed=8)
    tgt = torch.randint(0, V, (M,), device=DEV)
    tgt[::5] = -1
    out, lse = C.xent_fwd(logits, tgt, V)
    lr = logits.float()[:, :V].clone().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lr, tgt, ignore_index=-1)
    torch.testing.assert_close(out[0], ref.detach(), atol=1e-3, rtol=1e-3)
    ref.backward(torch.tensor(2.0, device=DEV))
    g = torch.tensor([2.0], device=DEV)
    dl = C.xent_bwd(logits, tgt, lse, g, out, V)
    _close(dl[:, :V], lr.grad, atol=2e-3)
    assert (dl[:, V:] == 0).all()


@pytest.mark.parametrize("M,V,ld,gs", [(40, 50257, 50304, 1.0), (33, 50257, 50304, 0.5),
                                       (9, 40000, 40064, 1.0), (5, 65536, 65536, 3.0)])
def test_cross_entropy_fused(M, V, ld, gs):
    """one-pass xent (loss + dlogits in forward, grad_out applied by xent_scale_) vs fp32 torch"""
    C = ext()
    logits = _bf(M, ld, scale=3.0, seed=9)
    tgt = torch.randint(0, V, (M,), device=DEV)
    tgt[::4] = -1
    tgt[1] = V - 1
    res = C.xent_fused(logits, tgt, V)
    assert res, "fused cross-entropy must cover this row width"
    out, dl = res
    lr = logits.float()[:, :V].clone().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lr, tgt, ignore_index=-1)
    torch.testing.assert_close(out[0], ref.detach(), atol=1e-3, rtol=1e-3)
    ref.backward(torch.tensor(gs, device=DEV))
    C.xent_scale_(dl, torch.tensor([gs], device=DEV))
    _close(dl[:, :V], lr.grad, atol=2e-3)
    assert (dl[:, V:] == 0).all()
    assert C.xent_fused(logits[:, :128].contiguous(), tgt, 100) == []  # outside the fused range


def test_adamw_matches_torch():
    C = ext()
    sizes = [1000, 37, 4096, 5]
    wds = [0.1, 0.0, 0.1, 0.0]
    n = sum(sizes)
    torch.manual_seed(0)
    master = torch.randn(n, device=DEV)
    grad = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    param = master.to(torch.bfloat16)
    # chunk table, chunk <= 1024 elements, never straddling a param
    starts, lens, cwd = [], [], []
    off = 0
    for s, wd in zip(sizes, wds):
        for c in range(0, s, 1024):
            starts.append(off + c)
            lens.append(min(1024, s - c))
            cwd.append(wd)
        off += s
    cs = torch.tensor(starts, device=DEV, dtype=torch.int64)
    cl = torch.tensor(lens, device=DEV, dtype=torch.int32)
    cw = torch.tensor(cwd, device=DEV, dtype=torch.float32)
    ref_params = [torch.nn.Parameter(t.clone()) for t in master.split(sizes)]
    opt = torch.optim.AdamW([{"params": [p], "weight_decay": wd} for p, wd in zip(ref_params, wds)],
                            lr=1e-3, betas=(0.9, 0.95))
    norm = torch.zeros(2, device=DEV)
    for step in range(1, 4):
        g = grad * step
        for p, gg in zip(ref_params, g.split(sizes)):
            p.grad = gg.clone()
        total = torch.nn.utils.clip_grad_norm_(ref_params, 1.0)
        opt.step()
        C.grad_sumsq(g, 1.0, norm)
        torch.testing.assert_close(norm[1], total, rtol=1e-4, atol=1e-4)
        C.adamw_step(cs, cl, cw, None, master, param, g, m, v, norm, 1e-3, 0.9, 0.95, 1e-8, step, 1.0, 1.0,
                     n, n)
    torch.testing.assert_close(master, torch.cat([p.detach() for p in ref_params]), atol=1e-5, rtol=1e-4)
    _close(param, master, atol=1e-2)


@pytest.mark.parametrize("gdtype", [torch.float32, torch.bfloat16])
def test_adamw_pieces_packed_moments(gdtype):
    """The ZeRO-1 form: the kernels update only some pieces of the flat buffers (a rank's slice of
    every bucket), the moments are packed (moment_start), the gradients may be the bf16 buffer a
    bf16 reduction left; grad_sumsq_chunks covers exactly those pieces.  Oracle: plain fp32 math."""
    from mingpt_distributed_amd.optim import make_chunk_table

    C = ext()
    torch.manual_seed(0)
    n = 200_000
    pieces = [(0, 40_000, 0.1, 0), (70_016, 140_032, 0.0, 40_000), (150_016, 199_936, 0.1, 110_016)]
    nm = sum(b - a for a, b, _, _ in pieces)
    t = make_chunk_table(pieces, DEV, n, nm)
    cs, cl, cw, cm = t.start, t.len, t.wd, t.mstart
    assert (t.end, t.mend) == (199_936, nm)
    master = torch.randn(n, device=DEV)
    param = master.to(torch.bfloat16)
    g = torch.randn(n, device=DEV).to(gdtype)
    m = torch.zeros(nm, device=DEV)
    v = torch.zeros(nm, device=DEV)
    ref_master, ref_m, ref_v = master.clone(), m.clone(), v.clone()
    norm = torch.zeros(2, device=DEV)
    lr, b1, b2, eps, gs, clip = 1e-3, 0.9, 0.95, 1e-8, 0.5, 1.0
    for step in range(1, 3):
        C.grad_sumsq_chunks(cs, cl, g, gs, norm, t.end)
        gf = g.float()
        sq = sum((gf[a:b] * gs).pow(2).sum() for a, b, _, _ in pieces)
        torch.testing.assert_close(norm[1], sq.sqrt(), rtol=1e-4, atol=1e-4)
        C.adamw_step(cs, cl, cw, cm, master, param, g, m, v, norm, lr, b1, b2, eps, step, gs, clip,
                     t.end, t.mend)
        coef = min(1.0, clip / (sq.sqrt().item() + 1e-6))
        for a, b, wd, ma in pieces:
            gg = gf[a:b] * gs * coef
            mm, vv = ref_m[ma:ma + b - a], ref_v[ma:ma + b - a]
            mm.mul_(b1).add_(gg, alpha=1 - b1)
            vv.mul_(b2).addcmul_(gg, gg, value=1 - b2)
            ref_master[a:b].mul_(1 - lr * wd)
            denom = vv.sqrt() / (1 - b2 ** step) ** 0.5 + eps
            ref_master[a:b].addcdiv_(mm, denom, value=-lr / (1 - b1 ** step))
    torch.testing.assert_close(master, ref_master, atol=1e-5, rtol=1e-4)  # untouched outside pieces
    torch.testing.assert_close(m, ref_m, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(v, ref_v, atol=1e-7, rtol=1e-4)
    with pytest.raises(ValueError):
        make_chunk_table([(0, n + 64, 0.0, None)], DEV, n)
    # a table validated against larger buffers than the ones handed in fails in the binding
    with pytest.raises(RuntimeError, match="chunk table"):
        C.grad_sumsq_chunks(cs, cl, g[:100_000], gs, norm, t.end)
    with pytest.raises(RuntimeError, match="chunk table"):
        C.adamw_step(cs, cl, cw, cm, master, param, g, m[:1000], v[:1000], norm, lr, b1, b2, eps, 3, gs,
                     clip, t.end, t.mend)


@pytest.mark.parametrize("N", [768, 2304, 3072, 520])  # 32- and 64-lane bias-grad row chunks
def test_elementwise(N):
    C = ext()
    M = 130
    x, b, r = _bf(M, N, seed=9), _bf(N, seed=10), _bf(M, N, seed=11)
    pre = torch.empty_like(x)
    y = C.bias_act(x, b, pre, 1)
    _close(pre, x.float() + b.float(), atol=2e-2)
    _close(y, R.gelu_tanh(x.float() + b.float()), atol=2e-2)
    dy = _bf(M, N, seed=12)
    xr = (x.float() + b.float()).requires_grad_()
    R.gelu_tanh(xr).backward(dy.float())
    _close(C.gelu_bwd(dy, pre), xr.grad, atol=3e-2)
    out = C.bias_dropout_residual(x, b, r, 0.0, 7)
    _close(out, r.float() + x.float() + b.float(), atol=3e-2)
    out = C.bias_dropout_residual(x, b, r, 0.5, 7)
    kept = (out.float() - r.float()).abs() > 1e-6
    assert abs(kept.float().mean().item() - 0.5) < 0.03
    dx = C.dropout_bwd(dy, 0.5, 7)
    assert ((dx.float() != 0) == kept).float().mean().item() > 0.99
    db = torch.zeros(N, device=DEV)
    C.bias_grad(dy, db)
    torch.testing.assert_close(db, dy.float().sum(0), atol=2e-2, rtol=1e-3)
    db2 = torch.zeros(N, device=DEV)
    dx2 = C.dropout_bias_grad(dy, db2, 0.5, 7)
    torch.testing.assert_close(dx2.float(), dx.float())
    torch.testing.assert_close(db2, dx.float().sum(0), atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("B,N,K", [(1, 2304, 768), (3, 768, 3072), (8, 50257, 768), (5, 100, 64)])
def test_gemv_epilogues(B, N, K):
    """Decode-time skinny GEMM (gemv.hip) vs fp32 torch for every epilogue."""
    C = ext()
    x, w, b = _bf(B, K, seed=21), _bf(N, K, scale=0.05, seed=22), _bf(N, seed=23)
    ref = x.float() @ w.float().t()
    ld = (N + 7) // 8 * 8
    y0 = C.gemv(x, w, 0, None, None, ld)
    _close(y0[:, :N], ref, atol=2e-2)
    _close(C.gemv(x, w, 1, b, None, 0), ref + b.float(), atol=2e-2)
    z = ref + b.float()
    _close(C.gemv(x, w, 2, b, None, 0), 0.5 * z * (1 + torch.tanh(0.7978845608 * (z + 0.044715 * z ** 3))),
           atol=2e-2)
    r = _bf(B, N, seed=24)
    _close(C.gemv(x, w, 3, b, r, 0), z + r.float(), atol=3e-2)
    # fused LayerNorm staging == layernorm_fwd then the plain skinny GEMM (same rounding points)
    lw, lb = _bf(K, seed=25) * 0.1 + 1, _bf(K, seed=26) * 0.1
    h, _, _ = C.layernorm_fwd(x, lw, lb, 1e-5)
    torch.testing.assert_close(C.gemv(x, w, 1, b, None, 0, lw, lb, 1e-5), C.gemv(h, w, 1, b, None, 0),
                               atol=1e-2, rtol=1e-2)
