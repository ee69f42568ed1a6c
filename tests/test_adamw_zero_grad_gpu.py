"""AdamW with the gradient zeroing fused into the update kernel (FusedAdamW.step(zero_grad=True),
what StepEngine runs): the grads are zero after the step, only the chunk table's elements are
written, and the update equals the unfused step."""
import pytest
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.ops._ext import ext
from mingpt_distributed_amd.optim import make_chunk_table
from mingpt_distributed_amd.trainer import StepEngine

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model():
    torch.manual_seed(0)
    return GPT(GPTConfig(n_layer=2, n_head=4, n_embed=128, vocab_size=300, block_size=64,
                         embed_drop=0.0, resid_drop=0.0, attn_drop=0.0), verbose=False)


def test_kernel_zeroes_exactly_the_table_and_matches_unfused():
    C = ext()
    n = 10000
    pieces = [(0, 4100, 0.1, None), (4104, 7001, 0.0, None), (7004, 9999, 0.1, None)]  # odd tails
    t = make_chunk_table(pieces, DEV, n)
    g = torch.Generator(device=DEV).manual_seed(3)
    master = torch.randn(n, device=DEV, generator=g)
    grad = torch.randn(n, device=DEV, generator=g)
    outs = []
    for fused in (False, True):
        mst, gr = master.clone(), grad.clone()
        prm = mst.to(torch.bfloat16)
        m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        norm = torch.zeros(2, device=DEV)
        C.grad_sumsq_chunks(t.start, t.len, gr, 1.0, norm, t.end)
        C.adamw_step(t.start, t.len, t.wd, None, mst, prm, gr, m, v, norm, 1e-3, 0.9, 0.95, 1e-8, 1, 1.0,
                     1.0, t.end, t.mend, gr if fused else None)
        outs.append((mst, prm, m, v, gr))
    for a, b in zip(outs[0][:4], outs[1][:4]):
        assert torch.equal(a, b)  # the zeroing does not change the update
    gz = outs[1][4]
    inside = torch.zeros(n, dtype=torch.bool, device=DEV)
    for a, b, _, _ in pieces:
        inside[a:b] = True
    assert gz[inside].abs().max().item() == 0.0
    assert torch.equal(gz[~inside], grad[~inside])  # padding between pieces untouched


def test_engine_step_leaves_zero_grads_and_trains():
    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=DEV)
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 300, (8, 64), generator=g)
    y = torch.roll(x, -1, 1)
    l0 = eng.train_step([(x, y)]).item()
    torch.cuda.synchronize()
    assert eng.store.grad.abs().max().item() == 0.0
    for _ in range(5):
        l1 = eng.train_step([(x, y)]).item()
    assert l1 < l0
    assert eng.store.grad.abs().max().item() == 0.0
