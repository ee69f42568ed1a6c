"""Weight gradients on the side stream (ops/streams.py) give the gradients of the in-order
backward: one StepEngine backward of the same weights and batch with the side stream off and on,
compared on the whole flat fp32 gradient buffer (split-K fp32 atomics may add in another order,
hence a tolerance rather than bit equality), and the side stream joined by the step."""
import copy

import pytest
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.ops import streams
from mingpt_distributed_amd.trainer import StepEngine

pytestmark = pytest.mark.gpu


def _grads(base, x, y, on):
    streams.set_enabled(on, "1")  # every weight gradient on the side stream, whatever its size
    try:
        eng = StepEngine(copy.deepcopy(base), lr=1e-3)
        eng.forward_backward(x, y)
        assert not streams.pending()  # forward_backward joined the side stream
        torch.cuda.synchronize()
        return eng.store.grad.clone()
    finally:
        streams.set_enabled(True, "auto")


@pytest.mark.parametrize("n_embed,n_head", [(256, 4), (768, 12)])
def test_side_stream_grads_match_in_order(n_embed, n_head):
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=3, n_head=n_head, n_embed=n_embed, vocab_size=2048, block_size=256,
                    embed_drop=0.0, resid_drop=0.0, attn_drop=0.0)
    base = GPT(cfg, verbose=False)
    x = torch.randint(0, 2048, (8, 256), device="cuda")
    y = torch.roll(x, -1, 1)
    g0 = _grads(base, x, y, False)
    g1 = _grads(base, x, y, True)
    assert torch.isfinite(g1).all()
    torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-6 * g0.abs().max().item())


def test_side_stream_training_steps_reduce_loss():
    streams.set_enabled(True, "1")
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=2, n_head=4, n_embed=256, vocab_size=1000, block_size=128,
                    embed_drop=0.1, resid_drop=0.1, attn_drop=0.1)
    eng = StepEngine(GPT(cfg, verbose=False), lr=1e-3)
    x = torch.randint(0, 1000, (8, 128), device="cuda")
    y = torch.roll(x, -1, 1)
    try:
        losses = [eng.train_step([(x, y)]).item() for _ in range(20)]
    finally:
        streams.set_enabled(True, "auto")
    assert losses[-1] < losses[0] - 1.0, losses


def test_auto_mode_picks_small_weight_gradients():
    streams.set_enabled(True, "auto")
    assert streams.use_for(16384) and not streams.use_for(32768) and not streams.use_for(131072)
