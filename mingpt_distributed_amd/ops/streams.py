"""Weight-gradient stream: the block weight gradients run beside the backward's critical path.

In a transformer block's backward only the data gradients (dgrad -> LayerNorm backward -> the
next block) are on the critical path; the four weight gradients (``main_grad += dY^T X``) feed
nothing but the all-reduce and the optimizer.  They are issued on a second HIP stream that waits
(stream-ordered, no host sync) for the compute stream at the point of issue, so each one runs
concurrently with the data-gradient GEMMs, the attention backward and the memory-bound LayerNorm /
dropout kernels after it: the hardware dispatcher fills CUs left idle by one kernel's last round of
tiles with the other's blocks (gpt2-xl's 175-tile weight gradients leave 81 of 256 CUs idle on their
own; the ~30 us elementwise kernels leave the matrix cores idle).

Ordering contract:
* :func:`run_wgrad` -- the side stream waits for everything the compute stream has issued so far,
  runs the GEMM, and the inputs are ``record_stream``'d so the caching allocator does not hand
  their memory out before the side stream is done with it.
* :func:`join` -- the compute stream waits for every weight gradient issued so far.  Called after
  ``loss.backward()`` (``StepEngine.forward_backward``) and by every reader of ``main_grad``
  (the data-parallel engines' ``finish``, the optimizer step).
* :func:`collective_stream` -- a gradient collective launched mid-backward is issued on the side
  stream (after it waits for the compute stream), so it is ordered after the weight gradients of
  its bucket without making the compute stream wait.

Only parameters that own a ``main_grad`` use the stream (their buffer is read after a join); a
gradient that autograd returns is computed in order.  ``MINGPT_WGRAD_STREAM=0`` runs everything
on the compute stream.  Replaces nothing in the reference: its DDP backward is one stream
(``/root/reference/mingpt/trainer.py:71``).
"""
from __future__ import annotations

import contextlib
import os
from typing import Callable, Dict

import torch

_ENABLED = os.environ.get("MINGPT_WGRAD_STREAM", "1") == "1"
_side: Dict[int, "torch.cuda.Stream"] = {}
_pending: set = set()


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    """Switch the side stream on / off (tests, A/B).  Joins first so nothing is left in flight."""
    global _ENABLED
    join()
    _ENABLED = bool(on)


def _stream(dev: torch.device) -> "torch.cuda.Stream":
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = _side[idx] = torch.cuda.Stream(device=idx)
    return s


def run_wgrad(fn: Callable[[], None], *inputs: torch.Tensor) -> None:
    """Run ``fn`` (a weight-gradient accumulation reading ``inputs``) on the side stream."""
    if not _ENABLED or not inputs[0].is_cuda:
        fn()
        return
    dev = inputs[0].device
    s = _stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    for t in inputs:
        t.record_stream(s)
    _pending.add(s.device.index)


def join() -> None:
    """The compute stream waits for every weight gradient issued so far (no host block)."""
    if not _pending:
        return
    for idx in list(_pending):
        torch.cuda.current_stream(idx).wait_stream(_side[idx])
    _pending.clear()


def pending() -> bool:
    return bool(_pending)


@contextlib.contextmanager
def collective_stream(device: torch.device):
    """Issue a mid-backward collective (and its wire conversion) on the side stream, ordered
    after the compute stream's kernels so far and after every weight gradient issued so far."""
    if not _pending or device.type != "cuda":
        yield
        return
    s = _stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        yield
