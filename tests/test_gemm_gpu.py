"""MFMA GEMM (csrc/kernels/gemm.hip) vs fp32 PyTorch, all layouts and epilogues, tail shapes."""
import pytest
import torch

from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=[0, 1, 5, 6], ids=["auto", "t128", "w4", "w4n192"])
def tile_config(request):
    """Run every GEMM test under each tile configuration of gemm.hip (0 = per-shape choice)."""
    from mingpt_distributed_amd.ops._ext import ext

    ext().gemm_set_variant(request.param)
    yield request.param
    ext().gemm_set_variant(0)


def _bf(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV, torch.bfloat16)


def _check(out, ref, K):
    tol = 2e-2 * (K ** 0.5) * 0.25 + 2e-2
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=2e-2)


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 768), (200, 72, 136), (1000, 2304, 768),
                                   (64, 16, 48)])
def test_nt_plain_bias(M, N, K):
    a, b, bias = _bf(M, K, seed=1), _bf(N, K, seed=2), _bf(N, seed=3)
    ref = a.float() @ b.float().t()
    _check(G.gemm_nt(a, b), ref, K)
    _check(G.gemm_nt(a, b, bias=bias, epi="bias"), ref + bias.float(), K)


def test_nt_identity_asymmetric():
    # A = I catches a transposed C write (guide §3: always A=I with asymmetric B)
    K = 128
    a = torch.eye(K, device=DEV, dtype=torch.bfloat16)
    b = torch.arange(K * K, device=DEV, dtype=torch.float32).reshape(K, K).remainder(97).to(torch.bfloat16)
    torch.testing.assert_close(G.gemm_nt(a, b).float(), b.float().t())


def test_nt_padded_ld_vocab():
    M, V, K, ld = 130, 1001, 64, 1008
    a, b = _bf(M, K, seed=4), _bf(V, K, seed=5)
    out = G.gemm_nt(a, b, ld=ld)
    assert out.shape == (M, ld)
    _check(out[:, :V], a.float() @ b.float().t(), K)


def test_nt_gelu_and_resid():
    M, N, K = 300, 256, 192
    a, b, bias, r = _bf(M, K, seed=6), _bf(N, K, seed=7), _bf(N, seed=8), _bf(M, N, seed=9)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    out = G.gemm_nt(a, b, bias=bias, epi="gelu", pre_out=pre)
    z = a.float() @ b.float().t() + bias.float()
    _check(pre, torch.func.grad(lambda t: R.gelu_tanh(t).sum())(z), K)  # GELU'(z) for the backward
    _check(out, R.gelu_tanh(z), K)
    out = G.gemm_nt(a, b, bias=bias, epi="resid", resid=r, p=0.0)
    _check(out, z + r.float(), K)
    # dropout mask must match the standalone dropout kernel (same Philox element mapping)
    out = G.gemm_nt(a, b, bias=bias, epi="resid", resid=r, p=0.3, seed=11)
    from mingpt_distributed_amd.ops._ext import ext
    ref = ext().bias_dropout_residual(G.gemm_nt(a, b), bias, r, 0.3, 11)
    _check(out, ref.float(), K)


@pytest.mark.parametrize("M,N,K,Kb", [(256, 768, 2304, 2304), (100, 64, 72, 72), (130, 256, 1008, 1001)])
def test_nn(M, N, K, Kb):
    a, b = _bf(M, K, seed=10), _bf(Kb, N, seed=11)
    if Kb < K:  # padded reduction (lm-head dgrad): A's extra columns are zero
        a[:, Kb:] = 0
    ref = a.float()[:, :Kb] @ b.float()
    _check(G.gemm_nn(a, b), ref, K)
    gd = _bf(M, N, seed=12)  # a stored GELU'
    _check(G.gemm_nn(a, b, epi="gelu_bwd", aux=gd), ref * gd.float(), K)


@pytest.mark.parametrize("Mr,N,K", [(256, 768, 768), (192, 72, 136), (1024, 2304, 64)])
def test_tn_acc(Mr, N, K):
    a, b = _bf(Mr, N, seed=13), _bf(Mr, K, seed=14)
    c = torch.randn(N, K, device=DEV)
    ref = c + a.float().t() @ b.float()
    G.gemm_tn_acc(a, b, c)
    _check(c, ref, Mr)


@pytest.mark.parametrize("Mr,N,K", [(8040, 4800, 1704), (16384, 4800, 1600)])
def test_tn_acc_xl_shapes(Mr, N, K):
    # gpt2-xl weight-gradient shapes that quantise badly onto 256 CUs as 256^2 tiles (133 tiles: the
    # auto choice is T128 here, see pick_config); partial M / N tiles and a partial last K-tile
    # (8040 % 64 = 40) in the first shape
    a, b = _bf(Mr, N, seed=30, scale=0.5), _bf(Mr, K, seed=31, scale=0.5)
    c = torch.randn(N, K, device=DEV)
    ref = c + a.float().t() @ b.float()
    G.gemm_tn_acc(a, b, c)
    _check(c, ref, Mr)


def test_tn_acc_nvalid():
    Mr, V, ld, K = 128, 1001, 1008, 64
    a, b = _bf(Mr, ld, seed=15), _bf(Mr, K, seed=16)
    c = torch.zeros(V, K, device=DEV)
    G.gemm_tn_acc(a, b, c, n_valid=V)
    _check(c, a.float()[:, :V].t() @ b.float(), Mr)


@pytest.mark.parametrize("R,C,ld", [(768, 2304, 768), (130, 72, 136), (1001, 64, 1008)])
def test_transpose_padded(R, C, ld):
    w = _bf(R, C, seed=17)
    t = G.transpose(w, ld)
    assert t.shape == (C, ld)
    torch.testing.assert_close(t[:, :R], w.t(), rtol=0, atol=0)
    assert (t[:, R:] == 0).all()


@pytest.mark.parametrize("M,Nout,Nin", [(1000, 2304, 768), (256, 768, 3072), (130, 1001, 64)])
def test_dgrad_nt(M, Nout, Nin):
    """dX = dY @ W through the NT path against W^T (padded reduction for the vocab case)."""
    ld = (Nout + 7) // 8 * 8
    dy = _bf(M, ld, seed=18)
    dy[:, Nout:] = 0
    w = _bf(Nout, Nin, seed=19)
    ref = dy.float()[:, :Nout] @ w.float()
    _check(G.gemm_dgrad(dy, w), ref, Nout)
    gd = _bf(M, Nin, seed=20)
    _check(G.gemm_dgrad(dy, w, epi="gelu_bwd", aux=gd), ref * gd.float(), Nout)


@pytest.mark.parametrize("M", [1000, 8192])  # partial tiles (T128 kernel) / the W4 kernel
@pytest.mark.parametrize("nt", [False, True])  # NN from the stored weight / NT against W^T
def test_dgrad_gelu_bwd_bias_grad(M, nt):
    """The GELU' dgrad epilogue also accumulates the output's column sums (fc bias gradient) in
    its LDS-staged form: the fp32 values before their bf16 rounding, so equal to the sums of the
    stored output up to that rounding noise."""
    Nout, Nin = 768, 3072
    dy, w, gd = _bf(M, Nout, seed=21), _bf(Nout, Nin, seed=22), _bf(M, Nin, seed=23)
    db = torch.ones(Nin, device=DEV)
    wt = G.transpose(w, Nout) if nt else None
    out = G.gemm_dgrad(dy, w, epi="gelu_bwd", aux=gd.contiguous(), dbias=db, wt=wt)
    ref = (dy.float() @ w.float()) * gd.float()
    _check(out, ref, Nout)
    tol = 6e-3 * out.float().pow(2).sum(0).max().item() ** 0.5 + 1e-2  # ~5 sigma of the rounding noise
    torch.testing.assert_close(db, 1 + out.float().sum(0), atol=tol, rtol=1e-3)


def test_row_chunked_launches_match(monkeypatch):
    """Operands past 4 GiB (GPT-2 logits beyond ~42k tokens per GPU) are launched in M-chunks:
    force tiny chunks and compare against single launches."""
    from mingpt_distributed_amd.ops import gemm as G

    torch.manual_seed(0)
    M, K, N = 1000, 192, 320
    r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
    a, w, bias = r(M, K), r(N, K), r(N)
    dy = r(M, N)
    ref_nt = G.gemm_nt(a, w, bias=bias, epi="bias")
    pre_ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref_gelu = G.gemm_nt(a, w, bias=bias, epi="gelu", pre_out=pre_ref)
    ref_nn = G.gemm_nn(dy, w)
    ref_tn = G.gemm_tn_acc(dy, a, torch.zeros(N, K, device="cuda"))
    monkeypatch.setattr(G, "_MAX_BYTES", 256 * 2 * max(K, N))  # 256-row chunks
    assert len(G._row_chunks(M, 2 * K, 2 * N)) == 4
    torch.testing.assert_close(G.gemm_nt(a, w, bias=bias, epi="bias"), ref_nt, atol=0, rtol=0)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(G.gemm_nt(a, w, bias=bias, epi="gelu", pre_out=pre), ref_gelu, atol=0, rtol=0)
    torch.testing.assert_close(pre, pre_ref, atol=0, rtol=0)
    torch.testing.assert_close(G.gemm_nn(dy, w), ref_nn, atol=0, rtol=0)
    torch.testing.assert_close(G.gemm_tn_acc(dy, a, torch.zeros(N, K, device="cuda")), ref_tn,
                               atol=1e-3, rtol=1e-4)


def test_operands_past_4gib_single_launch(monkeypatch):
    """Operands past 4 GiB (the GPT-2 logits and their gradient beyond ~42k tokens) run as ONE
    launch: every block's buffer descriptor starts at its own tile / split origin, split-K ranges
    stay below 4 GiB.  Equal to the row-chunked launches (each operand chunk < 4 GiB)."""
    torch.manual_seed(0)
    M, V, D = 43008, 50304, 768  # [M, V] bf16 = 4.33 GB
    h = (torch.randn(M, D, device=DEV) * 0.5).to(torch.bfloat16)
    w = (torch.randn(V, D, device=DEV) * 0.05).to(torch.bfloat16)
    logits = G.gemm_nt(h, w, ld=V)
    dl = (torch.randn(M, V, device=DEV) * 0.01).to(torch.bfloat16)
    dh = G.gemm_dgrad(dl, w)
    gw = torch.zeros(V, D, device=DEV)
    G.gemm_tn_acc(dl, h, gw)
    monkeypatch.setattr(G, "_MAX_BYTES", 0x7FFFFFFF)  # chunks of < 2 GiB rows: the old launches
    assert len(G._row_chunks(M, 2 * V)) > 1
    torch.testing.assert_close(logits, G.gemm_nt(h, w, ld=V), atol=0, rtol=0)
    torch.testing.assert_close(dh, G.gemm_dgrad(dl, w), atol=0, rtol=0)
    gw2 = torch.zeros(V, D, device=DEV)
    G.gemm_tn_acc(dl, h, gw2)
    torch.testing.assert_close(gw, gw2, atol=1e-3 * gw2.abs().max().item(), rtol=1e-3)  # split order
    # and the rows past 4 GiB really are read: the last 512 rows' logits against fp32 torch
    ref = h[-512:].float() @ w.float().t()
    torch.testing.assert_close(logits[-512:].float(), ref, atol=2e-2, rtol=2e-2)


def test_deleted_tile_configs_are_rejected(tile_config):
    """Only reachable configurations can be forced (2-4 were deleted in round 5)."""
    from mingpt_distributed_amd.ops._ext import ext

    for v in (2, 3, 4, 7):
        with pytest.raises(Exception):
            ext().gemm_set_variant(v)
    ext().gemm_set_variant(tile_config)


@pytest.mark.parametrize("M", [8192, 1000])
def test_fragment_ordered_gelu_plane(M, tile_config):
    """Epilogues 6 / 7: the fc forward writes GELU'(z) in the fragment order of the W4 256x256 tiles
    (no LDS staging for that plane) and the fc2 data gradient reads it in the same order.  y, the
    data gradient and its bias-gradient column sums equal the row-major epilogues 2 / 4 exactly
    (same products, same staging of the other plane); partial tiles (M = 1000) included."""
    Nin, Nout = 768, 3072
    x, w, b = _bf(M, Nin, seed=41), _bf(Nout, Nin, seed=42, scale=0.05), _bf(Nout, seed=43, scale=0.1)
    dz, wp = _bf(M, Nin, seed=44), _bf(Nin, Nout, seed=45, scale=0.05)
    pre = torch.empty(M, Nout, device=DEV, dtype=torch.bfloat16)
    y0 = G.gemm_nt(x, w, bias=b, epi="gelu", pre_out=pre)
    fr = torch.empty(G.frag_aux_elems(M, Nout), device=DEV, dtype=torch.bfloat16)
    y1 = G.gemm_nt(x, w, bias=b, epi="gelu", pre_out=fr, frag=True)
    if tile_config in (0, 5):  # the same W4-256 kernel on both sides: bitwise
        assert torch.equal(y1, y0)
        assert torch.equal(G.frag_plane_rowmajor(fr, M, Nout), pre)  # the documented order
    else:
        torch.testing.assert_close(y1, y0, atol=2e-2, rtol=2e-2)
    db0 = torch.zeros(Nout, device=DEV)
    db1 = torch.zeros(Nout, device=DEV)
    d0 = G.gemm_dgrad(dz, wp, epi="gelu_bwd", aux=pre, dbias=db0)
    d1 = G.gemm_dgrad(dz, wp, epi="gelu_bwd", aux=fr, dbias=db1, aux_frag=True)
    if tile_config in (0, 5):  # the same W4-256 kernel on both sides: bitwise
        assert torch.equal(d1, d0)
    ref = (dz.float() @ wp.float()) * pre.float()
    _check(d1, ref, Nin)
    tol = 6e-3 * d1.float().pow(2).sum(0).max().item() ** 0.5 + 1e-2
    torch.testing.assert_close(db1, d1.float().sum(0), atol=tol, rtol=1e-3)
