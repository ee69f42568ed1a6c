"""Causal flash attention (csrc/kernels/attention.hip) vs the fp32 PyTorch reference."""
import os

import pytest
import torch

from mingpt_distributed_amd.ops import reference as R
from mingpt_distributed_amd.ops._ext import ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=[1, 2], ids=["bwd_persistent", "bwd_partials"])
def bwd_mode(request):
    """Every test under both backward schedules: one workgroup per (b, h) summing dQ in place,
    and one workgroup per (key block, b, h) with dQ partials + a finalize pass."""
    ext().attention_set_bwd_mode(request.param)
    yield request.param
    ext().attention_set_bwd_mode(0)


def _split(qkv, B, T, H):
    D = qkv.shape[-1] // 3
    q, k, v = qkv.float().view(B, T, 3 * D).split(D, dim=2)
    f = lambda t: t.reshape(B, T, H, D // H).transpose(1, 2)
    return f(q), f(k), f(v)


@pytest.mark.parametrize("B,T,H,hd", [(2, 128, 3, 64), (1, 200, 2, 64), (2, 1024, 2, 64), (1, 777, 2, 64),
                                      (2, 520, 3, 64), (2, 256, 4, 32),
                                      (1, 96, 3, 16), (1, 64, 1, 64), (1, 300, 2, 128), (2, 200, 2, 96),
                                      (1, 520, 2, 80), (1, 130, 2, 48), (1, 200, 3, 8), (1, 777, 1, 24),
                                      (1, 256, 2, 112)])
def test_attention_fwd_bwd(B, T, H, hd):
    C = ext()
    torch.manual_seed(0)
    D = H * hd
    qkv = torch.randn(B * T, 3 * D, device=DEV).to(torch.bfloat16)
    out, lse, mask = C.attention_fwd(qkv, B, T, H, 0.0, 0)
    qkv_r = qkv.float().requires_grad_()
    q, k, v = _split(qkv_r, B, T, H)
    ref = R.causal_attention(q, k, v, 0.0, False).transpose(1, 2).reshape(B * T, D)
    torch.testing.assert_close(out.float(), ref.detach(), atol=2e-2, rtol=2e-2)
    # lse (log2 domain) vs reference
    s = (q @ k.transpose(-1, -2)) / hd ** 0.5
    s = s.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=DEV).tril(), float("-inf"))
    lse_ref = torch.logsumexp(s, -1) / torch.log(torch.tensor(2.0))
    torch.testing.assert_close(lse.view(B, H, T), lse_ref.detach(), atol=2e-2, rtol=1e-3)
    dout = torch.randn(B * T, D, device=DEV).to(torch.bfloat16)
    ref.backward(dout.float())
    dqkv = C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, 0.0, 0)
    g = qkv_r.grad
    scale = g.abs().max().item()
    torch.testing.assert_close(dqkv.float(), g, atol=3e-2 * max(1.0, scale / 4), rtol=5e-2)


@pytest.mark.parametrize("B,T,H,hd,p", [(2, 1024, 2, 64, 0.0), (2, 1024, 2, 64, 0.1), (1, 520, 2, 80, 0.0),
                                        (1, 300, 2, 128, 0.1), (2, 200, 2, 96, 0.0), (1, 777, 1, 24, 0.0),
                                        (2, 128, 3, 64, 0.0)])
def test_attention_bwd_fused_bias_grad(B, T, H, hd, p):
    """attention_bwd(..., dbias) adds the column sums of dqkv (the qkv bias gradient) into dbias:
    fused into the key-block kernel (dK / dV) and the dQ finalize (dQ), or a separate pass in the
    persistent schedule.  Equal to the sums of the returned dqkv, and dqkv itself unchanged."""
    C = ext()
    torch.manual_seed(1)
    D = H * hd
    qkv = torch.randn(B * T, 3 * D, device=DEV).to(torch.bfloat16)
    out, lse, mask = C.attention_fwd(qkv, B, T, H, p, 7)
    dout = torch.randn(B * T, D, device=DEV).to(torch.bfloat16)
    plain = C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, p, 7)
    db = torch.full((3 * D,), 0.5, device=DEV)
    dqkv = C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, p, 7, db)
    torch.testing.assert_close(dqkv, plain, atol=0, rtol=0)
    ref = 0.5 + dqkv.float().sum(0)
    # dQ / dK / dV are summed before their bf16 rounding (independent errors of <= 2^-9 relative
    # per element): ~6 sigma of that rounding noise over the column
    tol = 6e-3 * dqkv.float().pow(2).sum(0).max().item() ** 0.5 + 1e-2
    torch.testing.assert_close(db, ref, atol=tol, rtol=2e-3)


@pytest.mark.parametrize("B,T,H,p", [(2, 1024, 2, 0.1), (1, 777, 2, 0.1), (1, 520, 3, 0.0), (3, 1000, 1, 0.1),
                                     (1, 257, 2, 0.1), (2, 2048, 1, 0.1)])
def test_attention_bwd64_matches_general_kernel(B, T, H, p, bwd_mode):
    """hd = 64 key-block backward (attn_bwd64_kernel: one wave per SIMD, pipelined units, causal mask
    in the accumulator init) against the general kernel it replaces (attn_bwd_kernel<4, 8>): the
    same products in the same order, so dQ / dK / dV agree bitwise; the fused qkv bias gradient up
    to the order of its cross-workgroup atomics."""
    C = ext()
    torch.manual_seed(3)
    D = H * 64
    qkv = torch.randn(B * T, 3 * D, device=DEV).to(torch.bfloat16)
    out, lse, mask = C.attention_fwd(qkv, B, T, H, p, 11)
    dout = torch.randn(B * T, D, device=DEV).to(torch.bfloat16)
    res = {}
    try:
        for on in (1, 0):
            C.attention_set_bwd64(on)
            db = torch.zeros(3 * D, device=DEV)
            res[on] = (C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, p, 11, db), db)
    finally:
        C.attention_set_bwd64(int(os.environ.get("MINGPT_ATTN_BWD64", "1")))
    assert torch.equal(res[1][0], res[0][0])
    torch.testing.assert_close(res[1][1], res[0][1], atol=1e-3, rtol=1e-4)


def test_attention_causality():
    """Perturbing token j must not change outputs at positions < j (reference defect D4)."""
    C = ext()
    B, T, H, hd = 1, 256, 2, 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).to(torch.bfloat16)
    out1 = C.attention_fwd(qkv, B, T, H, 0.0, 0)[0]
    qkv2 = qkv.clone()
    qkv2[200:] += 1.0
    out2 = C.attention_fwd(qkv2, B, T, H, 0.0, 0)[0]
    assert torch.equal(out1[:200], out2[:200])
    assert not torch.equal(out1[200:], out2[200:])


def test_attention_dropout_deterministic():
    C = ext()
    B, T, H, hd = 2, 256, 2, 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).to(torch.bfloat16)
    o1, l1, m1 = C.attention_fwd(qkv, B, T, H, 0.1, 42)
    o2, _, m2 = C.attention_fwd(qkv, B, T, H, 0.1, 42)
    o3, _, _ = C.attention_fwd(qkv, B, T, H, 0.1, 43)
    o0, l0, _ = C.attention_fwd(qkv, B, T, H, 0.0, 0)
    assert torch.equal(o1, o2) and not torch.equal(o1, o3)
    torch.testing.assert_close(l1, l0)  # softmax statistics use the undropped P
    dout = torch.randn_like(o1)
    d1 = C.attention_bwd(qkv, o1, dout, l1, m1, B, T, H, 0.1, 42)
    d2 = C.attention_bwd(qkv, o1, dout, l1, m2, B, T, H, 0.1, 42)
    # every gradient is register / workgroup-accumulated (no atomics): bitwise reproducible
    assert torch.equal(d1, d2) and torch.isfinite(d1.float()).all()


def test_attention_dropout_gradient_directional():
    """Directional derivative check of the dropout path: the same seed makes f deterministic."""
    C = ext()
    B, T, H, hd = 1, 128, 2, 64
    torch.manual_seed(1)
    qkv = (torch.randn(B * T, 3 * H * hd, device=DEV) * 0.5).to(torch.bfloat16)
    w = torch.randn(B * T, H * hd, device=DEV)
    o, lse, msk = C.attention_fwd(qkv, B, T, H, 0.2, 7)
    d = C.attention_bwd(qkv, o, w.to(torch.bfloat16), lse, msk, B, T, H, 0.2, 7).float()
    delta = torch.randn_like(qkv.float())
    eps = 0.05
    fp = (C.attention_fwd((qkv.float() + eps * delta).to(torch.bfloat16), B, T, H, 0.2, 7)[0].float() * w).sum()
    fm = (C.attention_fwd((qkv.float() - eps * delta).to(torch.bfloat16), B, T, H, 0.2, 7)[0].float() * w).sum()
    fd = (fp - fm) / (2 * eps)
    an = (d * delta).sum()
    assert abs(fd.item() - an.item()) < 0.08 * abs(an.item()) + 1.0


def _dense_keep(mask, B, T, H):
    """Dense [B, H, T(query), T(key)] keep matrix from the keep-bit row words (layout and bit
    order: attention_fwd.hip attn_dropmask_kernel; words of tiles past the diagonal are
    unspecified)."""
    ntw = 2 * ((T + 63) // 64)
    words = mask.view(B * H, ntw, T).to(torch.int64) & 0xFFFFFFFF  # [bh, j, q]
    key = torch.arange(T, device=mask.device)
    kk = key % 64
    j = (key // 64) * 2 + ((kk >> 2) & 1)
    e = 16 * (kk >> 5) + 4 * ((kk >> 3) & 3) + (kk & 3)  # the forward lane's value index
    bit = 16 * (e & 1) + (e >> 1)  # attn_common.h drop_bit: packed pair e >> 1
    w = words[:, j, :]  # [bh, key, q]
    return ((w >> bit[None, :, None]) & 1).transpose(1, 2).reshape(B, H, T, T).float()


@pytest.mark.parametrize("hd", [8, 16, 24, 32, 48, 64, 80, 96, 112, 128])
def test_attention_fwd_head_dims(hd):
    """Forward for every head dim the kernels take (multiples of 8 up to 128; hd > 64 uses two
    64-column LDS halves), with and without dropout, vs the fp32 reference (exact keep mask)."""
    C = ext()
    B, T, H = 2, 200, 2
    torch.manual_seed(hd)
    D = H * hd
    qkv = torch.randn(B * T, 3 * D, device=DEV).to(torch.bfloat16)
    q, k, v = _split(qkv, B, T, H)
    att = (q @ k.transpose(-1, -2)) / hd ** 0.5
    att = att.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=DEV).tril(), float("-inf"))
    for p in (0.0, 0.1):
        out, lse, mask = C.attention_fwd(qkv, B, T, H, p, 5)
        keep = _dense_keep(mask, B, T, H) * (65536.0 / (65536 - round(p * 65536))) if p > 0 else 1.0
        ref = ((att.softmax(-1) * keep) @ v).transpose(1, 2).reshape(B * T, D)
        torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2, msg=lambda m: f"p={p}: {m}")
        lse_ref = torch.logsumexp(att, -1) / torch.log(torch.tensor(2.0))
        torch.testing.assert_close(lse.view(B, H, T), lse_ref, atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("T", [128, 320, 512, 1024])
def test_attention_dropout_exact(T):
    """Forward and backward with dropout vs an fp32 reference that uses the kernel's exact mask."""
    C = ext()
    B, H, hd, p = 2, 2, 64, 0.1
    torch.manual_seed(3)
    D = H * hd
    qkv = torch.randn(B * T, 3 * D, device=DEV).to(torch.bfloat16)
    out, lse, mask = C.attention_fwd(qkv, B, T, H, p, 11)
    thr = round(p * 65536)
    keep = _dense_keep(mask, B, T, H) * (65536.0 / (65536 - thr))
    qkv_r = qkv.float().requires_grad_()
    q, k, v = _split(qkv_r, B, T, H)
    att = (q @ k.transpose(-1, -2)) / hd ** 0.5
    att = att.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=DEV).tril(), float("-inf")).softmax(-1)
    ref = ((att * keep) @ v).transpose(1, 2).reshape(B * T, D)
    torch.testing.assert_close(out.float(), ref.detach(), atol=3e-2, rtol=3e-2)
    dout = torch.randn(B * T, D, device=DEV).to(torch.bfloat16)
    ref.backward(dout.float())
    dqkv = C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, p, 11)
    g = qkv_r.grad
    scale = g.abs().max().item()
    torch.testing.assert_close(dqkv.float(), g, atol=3e-2 * max(1.0, scale / 4), rtol=5e-2)


@pytest.mark.parametrize("p", [0.1, 0.6])  # thr <= 0x8000 and > 0x8000: both SWAR keep tests
def test_attention_dropout_keep_rate(p):
    """The forward's counter-hash dropout keeps 1 - p of the causal entries (16-bit decisions: p is
    exact to 1/65536), uniformly over heads; >= 1e7 draws at the bench shape's head dim."""
    C = ext()
    B, T, H, hd = 4, 1024, 8, 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).to(torch.bfloat16)
    _, _, mask = C.attention_fwd(qkv, B, T, H, p, 5)
    keep = _dense_keep(mask, B, T, H)
    causal = torch.ones(T, T, dtype=torch.bool, device=DEV).tril()
    kc = keep[..., causal]
    assert kc.numel() >= 10_000_000
    rate = kc.mean().item()
    assert abs(rate - (1 - p)) < 0.001, rate
    # no structure across heads / rows: per-head rates agree
    per_head = keep[..., causal].mean(-1).flatten()
    assert (per_head - rate).abs().max().item() < 0.01
    _, _, mask2 = C.attention_fwd(qkv, B, T, H, p, 6)
    assert (keep != _dense_keep(mask2, B, T, H))[..., causal].float().mean().item() > 0.1  # seed matters



@pytest.mark.parametrize("hd", [64, 128, 24])
def test_attention_decode_split_keys(hd, bwd_mode):
    """Split-key decode attention (workgroups over key ranges, last one combines) vs fp32
    softmax(q K^T) V over keys 0..pos, with this step's K/V appended at row pos; repeated calls
    (the per-(b, h) counters must come back to zero)."""
    C = ext()
    B, H, Tmax = 3, 2, 700
    D = H * hd
    torch.manual_seed(hd)
    cache = torch.randn(B, Tmax, 3 * D, device=DEV).to(torch.bfloat16)
    for pos in (0, 63, 64, 500, 699, 64):
        qkv = torch.randn(B, 3 * D, device=DEV).to(torch.bfloat16)
        c = cache.clone()
        out = C.attention_decode(qkv, c, H, pos)
        assert torch.equal(c[:, pos, D:], qkv[:, D:])  # K/V appended
        q = qkv[:, :D].float().view(B, H, hd)
        k = c[:, :pos + 1, D:2 * D].float().view(B, pos + 1, H, hd)
        v = c[:, :pos + 1, 2 * D:].float().view(B, pos + 1, H, hd)
        att = torch.einsum("bhd,bthd->bht", q, k) / hd ** 0.5
        ref = torch.einsum("bht,bthd->bhd", att.softmax(-1), v).reshape(B, D)
        torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
