"""Main-grad protocol shared by the fused ops and the data-parallel engine.

Every parameter the engine manages carries ``p.main_grad``: an fp32 view into ONE flat gradient
buffer.  The GPU backward kernels accumulate weight gradients straight into it (the GEMM /
LayerNorm / embedding backward write fp32, no bf16 round trip, no extra copy pass), and return
``None`` to autograd for that input.  Readiness for the bucketed all-reduce is tracked by use
counts: a forward that consumes ``p`` calls :func:`note_use`, the matching backward calls
:func:`grad_done`; the engine launches a bucket's all-reduce when every use of every parameter in
it has produced its gradient.  (Tied weights such as ``wte``/``lm_head`` have two uses.)

Parameters without ``main_grad`` (e.g. a model used outside the engine) get ordinary autograd
gradients from the same ops.
"""
from __future__ import annotations

import torch


def main_grad(p: torch.Tensor):
    return getattr(p, "main_grad", None)


def before_use(*params: torch.Tensor) -> None:
    """Call before launching kernels that read ``params``: under ZeRO-1 the compute stream waits
    (stream-ordered, no host block) for the all-gather that brings those weights up to date, so
    the gather of later layers overlaps the forward of earlier ones."""
    for p in params:
        eng = getattr(p, "_mg_engine", None)
        if eng is not None:
            eng.before_use(p)


def note_use(p: torch.Tensor) -> None:
    """Count one use of ``p`` whose gradient the coming backward will produce.  Call it where
    the caller's grad mode is in force (``fused._EngineFn.run``), never inside
    ``autograd.Function.forward`` (grad mode is always off there)."""
    eng = getattr(p, "_mg_engine", None)
    if eng is not None and p.requires_grad:
        eng.note_use(p)


def grad_done(p: torch.Tensor) -> None:
    eng = getattr(p, "_mg_engine", None)
    if eng is not None:
        eng.grad_done(p)


def grad_target(p: torch.Tensor):
    """fp32 buffer to accumulate ``p``'s gradient into; a fresh zero buffer if no main_grad."""
    mg = main_grad(p)
    if mg is not None:
        return mg, True
    return torch.zeros(p.shape, dtype=torch.float32, device=p.device), False


def finish(p: torch.Tensor, buf: torch.Tensor, is_main: bool):
    """Return value for autograd: None when accumulated into main_grad, else the gradient."""
    if is_main:
        grad_done(p)
        return None
    return buf.to(p.dtype)
