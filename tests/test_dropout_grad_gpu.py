"""Model-level gradients with dropout ON, on the GPU path (hand-written kernels end to end).

The flagship bench trains at p = 0.1 at all four dropout sites of the reference
(/root/reference/mingpt/model.py:140 embedding, :150 attention probabilities, :183 and :215 the
residual branches).  Their masks are counter hashes regenerated in the backward, and block l's MLP
residual-dropout backward runs inside its consumer's LayerNorm backward (ops/fused.py DropLink:
block l+1's ln_1, or ln_f in HeadLossFn / HeadFn).  A seed or link mix-up there still trains, so
these tests pin the gradients themselves at GPT-2 width (D = 768, H = 12, V = 50257), 3 layers,
T = 256:

(a) directional derivatives: with every mask fixed by torch.manual_seed, the central difference
    of the loss along each parameter group's own gradient direction matches <grad, delta>;
(b) hand-off vs no hand-off: the same seeds with GPT.dropout_handoff = False (every block runs its
    own dropout_bias_grad pass) give the same flat gradient, for HeadLossFn and for HeadFn;
(c) hipGraph vs eager: replays of a captured forward + backward (dropout seeds offset by the
    in-graph counter, common.h eff_seed) against eager steps run with the same effective seeds.
"""
import pytest
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.ops import streams
from mingpt_distributed_amd.ops._ext import ext
from mingpt_distributed_amd.trainer import StepEngine

pytestmark = pytest.mark.gpu

B, T, L, V, P = 8, 256, 3, 50257, 0.1
SEED = 1234


def _engine(handoff=True):
    torch.manual_seed(0)
    m = GPT(GPTConfig(n_layer=L, n_head=12, n_embed=768, vocab_size=V, block_size=T, embed_drop=P,
                      resid_drop=P, attn_drop=P), verbose=False)
    m.dropout_handoff = handoff
    eng = StepEngine(m, lr=0.0, weight_decay=0.0, grad_clip=0.0, device=torch.device("cuda", 0))
    eng.model.train()
    return eng


@pytest.fixture(scope="module")
def data():
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, V, (B, T), generator=g)
    y = torch.randint(0, V, (B, T), generator=g)
    y[0, :5] = -1
    return x.cuda(), y.cuda()


@pytest.fixture(scope="module")
def eng():
    return _engine()


def _grads(eng, x, y, seed=SEED):
    eng.store.zero_grad()
    torch.manual_seed(seed)
    loss = eng.forward_backward(x, y).item()
    torch.cuda.synchronize()
    return loss, eng.store.grad.clone()


def _loss(eng, x, y, seed=SEED):
    torch.manual_seed(seed)  # the same masks as the gradient run
    with torch.no_grad():
        _, loss = eng.model(x, y)
    return loss.item()


def _assert_grads_close(store, got, want, tol):
    bad = []
    for name, o, n in zip(store.names, store.offsets, store.numels):
        a, b = got[o:o + n], want[o:o + n]
        scale = b.abs().max().item() + 1e-30
        err = (a - b).abs().max().item() / scale
        if not err < tol:
            bad.append(f"{name}: max rel err {err:.2e}")
    assert not bad, "; ".join(bad)


GROUPS = {
    # block 0's MLP dropout backward runs in block 1's ln_1 backward (DropLink)
    "mlp_proj_0": ["transformer.h.0.mlp.c_proj.weight", "transformer.h.0.mlp.c_proj.bias"],
    # the last block's runs in ln_f's (HeadLossFn)
    "mlp_proj_last": [f"transformer.h.{L - 1}.mlp.c_proj.weight", f"transformer.h.{L - 1}.mlp.c_proj.bias"],
    # attention-branch dropout backward fused into ln_2's; attention-probability dropout
    "attn_1": ["transformer.h.1.attn.c_attn.weight", "transformer.h.1.attn.c_attn.bias",
               "transformer.h.1.attn.c_proj.weight", "transformer.h.1.attn.c_proj.bias"],
    "mlp_fc_1": ["transformer.h.1.mlp.c_fc.weight", "transformer.h.1.mlp.c_fc.bias",
                 "transformer.h.1.ln_2.weight", "transformer.h.1.ln_2.bias"],
    # everything upstream of every mask, plus the embedding dropout
    "embedding": ["transformer.wpe.weight", "transformer.h.0.ln_1.weight", "transformer.h.0.ln_1.bias"],
}


@pytest.mark.parametrize("group", list(GROUPS))
def test_directional_derivative_with_dropout(eng, data, group):
    """(f(w + d+) - f(w + d-)) = <grad, d+ - d->, d+- = bf16(w +- eps g_group) - w: the
    perturbation is taken after the bf16 rounding of the compute weights, so the linear term is
    exact and eps only has to keep the second-order residue small."""
    x, y = data
    s = eng.store
    _, g = _grads(eng, x, y)
    d = torch.zeros_like(g)
    for name in GROUPS[group]:
        i = s.by_name[name]
        o, n = s.offsets[i], s.numels[i]
        d[o:o + n] = g[o:o + n]
    gg = (d * d).sum().item()
    assert gg > 0, group
    eps = 0.01 / gg  # predicted loss change 2 eps |g|^2 = 0.02
    base = s.flat.clone()
    plus = (base.float() + eps * d).to(torch.bfloat16)
    minus = (base.float() - eps * d).to(torch.bfloat16)
    pred = (g.double() * (plus.double() - minus.double())).sum().item()
    try:
        s.flat.copy_(plus)
        fp = _loss(eng, x, y)
        s.flat.copy_(minus)
        fm = _loss(eng, x, y)
    finally:
        s.flat.copy_(base)
    got = fp - fm
    assert abs(got - pred) < 0.03 * abs(pred), f"{group}: finite difference {got:.5f} vs <grad, delta> {pred:.5f}"


def test_handoff_matches_unfused_dropout_backward(eng, data):
    """Loss head (HeadLossFn): the DropLink hand-off and the per-block dropout_bias_grad fallback
    see the same masks, so the flat gradients agree up to fp32 atomic summation order."""
    x, y = data
    la, ga = _grads(eng, x, y)
    plain = _engine(handoff=False)
    lb, gb = _grads(plain, x, y)
    assert abs(la - lb) <= 1e-6 * abs(la)
    _assert_grads_close(eng.store, ga, gb, tol=2e-3)
    # a different seed draws different masks: the comparison is not vacuous
    _, gc = _grads(plain, x, y, seed=SEED + 1)
    i = eng.store.by_name["transformer.h.0.mlp.c_proj.bias"]
    o, n = eng.store.offsets[i], eng.store.numels[i]
    assert (gc[o:o + n] - ga[o:o + n]).abs().max() > 0.05 * ga[o:o + n].abs().max()
    del plain


def test_handoff_matches_unfused_logits_head(data):
    """The same through HeadFn (logits only, a custom loss on them): ln_f's backward takes the
    last block's hand-off there too."""
    x, _ = data
    r = torch.randn(B, T, V, generator=torch.Generator().manual_seed(9)).to("cuda", torch.bfloat16)

    def run(handoff):
        e = _engine(handoff)
        e.store.zero_grad()
        torch.manual_seed(SEED)
        logits, _ = e.model(x)
        (logits.float() * r.float()).sum().mul(1e-3).backward()
        streams.join()
        torch.cuda.synchronize()
        return e.store, e.store.grad.clone()

    store, ga = run(True)
    _, gb = run(False)
    _assert_grads_close(store, ga, gb, tol=2e-3)


def test_hipgraph_replay_matches_eager_with_dropout(eng, data):
    x, y = data
    C = ext()
    dev = eng.device
    seed_buf = torch.zeros(1, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):  # warm-up off the capture stream, as torch.cuda.graph requires
        for _ in range(2):
            eng.forward_backward(x, y)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    rng = torch.get_rng_state()  # the seeds the capture draws
    graph = torch.cuda.CUDAGraph()
    C.set_graph_state(seed_buf, None)
    try:
        with torch.cuda.graph(graph):
            seed_buf.add_(1)
            loss_buf = eng.forward_backward(x, y)
    finally:
        C.set_graph_state(None, None)
    replays = []
    for _ in range(2):
        eng.store.zero_grad()
        graph.replay()
        torch.cuda.synchronize()
        replays.append((loss_buf.item(), eng.store.grad.clone()))
    assert replays[0][0] != replays[1][0]  # each replay draws new masks
    for k in range(2):  # eager steps with the same effective seeds: counter k + 1
        torch.set_rng_state(rng)
        seed_buf.fill_(k + 1)
        C.set_graph_state(seed_buf, None)
        try:
            eng.store.zero_grad()
            le = eng.forward_backward(x, y).item()
        finally:
            C.set_graph_state(None, None)
        torch.cuda.synchronize()
        assert abs(le - replays[k][0]) <= 1e-5 * abs(le), (k, le, replays[k][0])
        _assert_grads_close(eng.store, eng.store.grad, replays[k][1], tol=2e-3)
    del graph
