"""Gradient-readiness protocol (ops/grads.py): a parameter use is counted in the CALLER's grad
mode (inside autograd.Function.forward grad mode is always off), so a tied weight used twice is
ready only after its second gradient -- never after the first."""
import torch

from mingpt_distributed_amd.ops.fused import _EngineFn
from mingpt_distributed_amd.ops.grads import finish


class _Eng:
    def __init__(self):
        self.uses, self.ready = 0, 0

    def before_use(self, p):
        pass

    def note_use(self, p):
        self.uses += 1

    def grad_done(self, p):
        self.uses -= 1
        if self.uses <= 0:
            self.ready += 1


class _Mul(_EngineFn):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return x * w

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        ctx.w.main_grad.add_((g * x).sum(0))
        return g * ctx.w, finish(ctx.w, ctx.w.main_grad, True)


def test_tied_weight_ready_after_its_last_gradient():
    w = torch.nn.Parameter(torch.ones(4))
    w.main_grad = torch.zeros(4)
    w._mg_engine = eng = _Eng()
    x = torch.randn(3, 4, requires_grad=True)
    y = _Mul.run(_Mul.run(x, w), w)  # two uses of one weight (like wte in embedding + LM head)
    assert eng.uses == 2
    y.sum().backward()
    assert eng.ready == 1 and eng.uses == 0  # ready once, after both gradients
    with torch.no_grad():  # inference: no use counted, no backward owed
        _Mul.run(x, w)
    assert eng.uses == 0
