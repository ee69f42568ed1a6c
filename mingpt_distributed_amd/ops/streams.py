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
* :func:`run_wgrad` -- the side stream waits for everything the compute stream has issued so far
  and runs the GEMM.  The inputs' lifetime is bounded by a LAGGED join instead of
  ``record_stream``: the compute stream waits for weight gradient k - LAG (an event, usually long
  complete) before weight gradient k is issued, and only then are that one's inputs released, so
  the caching allocator can hand their memory to later compute-stream work at once.
  (``record_stream`` made every freed activation unusable until the CPU -- which runs a whole
  backward ahead of the GPU -- saw its event complete: at B = 128 the allocator grew instead of
  reusing, 600-720 ms per step against 127.)
* :func:`join` -- the compute stream waits for every weight gradient issued so far.  Called after
  ``loss.backward()`` (``StepEngine.forward_backward``) and by every reader of ``main_grad``
  (the data-parallel engines' ``finish``, the optimizer step).
* :func:`collective_stream` -- a gradient collective launched mid-backward is issued on the side
  stream (after it waits for the compute stream), so it is ordered after the weight gradients of
  its bucket without making the compute stream wait.

Only parameters that own a ``main_grad`` use the stream (their buffer is read after a join); a
gradient that autograd returns is computed in order.  ``MINGPT_WGRAD_STREAM``: ``auto`` (default;
small weight gradients only, see ``_MODE``), ``1`` always, ``0`` never.  Replaces nothing in the reference: its DDP backward is one stream
(``/root/reference/mingpt/trainer.py:71``).
"""
from __future__ import annotations

import contextlib
import os
from collections import deque
from typing import Callable, Deque, Dict, Optional, Tuple

import torch

# "auto" (default): the side stream for weight gradients over at most _AUTO_TOKENS rows (tokens),
# where their tiles underfill the GPU -- measured on one box each (profiles/round4_wgrad_stream_ab.txt):
# gpt2-xl at 16k tokens +1.2 %, at 32k tokens -3.3 %, GPT-2 at 131k tokens -1.1 % (those weight
# gradients fill the chip already; the concurrency only adds contention).  "1" always, "0" never.
_MODE = os.environ.get("MINGPT_WGRAD_STREAM", "auto").lower()
_ENABLED = _MODE != "0"
_AUTO_TOKENS = int(os.environ.get("MINGPT_WGRAD_STREAM_TOKENS", "16384"))
# ... and for models at least this wide (the weight gradients' smaller dimension): below it the
# GEMMs are launch-bound and the stream hand-offs cost more than the overlap gives (gpt-mini,
# D = 192: hipGraph step 4.73M tok/s single-stream vs 4.39M with the side stream,
# profiles/round6_compute_priority_ab.txt)
_AUTO_WIDTH = int(os.environ.get("MINGPT_WGRAD_STREAM_WIDTH", "512"))
# weight gradients in flight before the compute stream waits for the oldest (4 = one block)
_LAG = max(1, int(os.environ.get("MINGPT_WGRAD_LAG", "4")))
_side: Dict[int, "torch.cuda.Stream"] = {}
_inflight: Dict[int, Deque[Tuple["torch.cuda.Event", tuple]]] = {}
_pending: set = set()


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool, mode: str = "1") -> None:
    """Switch the side stream on (``mode`` "1": every weight gradient, "auto": small ones) or off
    (tests, A/B).  Joins first so nothing is left in flight."""
    global _ENABLED, _MODE
    join()
    _ENABLED = bool(on)
    _MODE = mode if on else "0"


def use_for(tokens: int, width: Optional[int] = None) -> bool:
    """Whether a weight gradient over ``tokens`` rows goes to the side stream."""
    return _ENABLED and (_MODE != "auto" or (tokens <= _AUTO_TOKENS and (width is None or width >= _AUTO_WIDTH)))


# HIP stream priority of the side stream (MINGPT_WGRAD_PRIORITY; lower = higher priority, 0 the
# default) and of the compute stream the engine runs forward + backward on
# (MINGPT_COMPUTE_PRIORITY): "auto" (default) = high (-1) whenever the side stream is in use for
# the batch, "off" = the caller's current stream, an integer = always that priority.  The
# dispatcher prefers the higher-priority queue's workgroups when a CU frees, so the critical
# path's kernels (LayerNorm backward, data gradients) stop waiting behind side-stream weight-
# gradient tiles: gpt2-xl B = 16 +3.3 %, 92.5k / 91.7k vs 89.2k / 89.1k tok/s on one box
# (profiles/round6_compute_priority_ab.txt); no change where the side stream is off
_SIDE_PRIO = int(os.environ.get("MINGPT_WGRAD_PRIORITY", "0"))
_COMPUTE_PRIO = os.environ.get("MINGPT_COMPUTE_PRIORITY", "auto").lower()
_compute: Dict[Tuple[int, int], "torch.cuda.Stream"] = {}


def _stream(dev: torch.device) -> "torch.cuda.Stream":
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = _side[idx] = torch.cuda.Stream(device=idx, priority=_SIDE_PRIO)
    return s


def compute_priority(tokens: int, width: Optional[int] = None):
    """The compute stream's priority for a batch of ``tokens`` rows of a model ``width`` wide
    (None: the current stream)."""
    if _COMPUTE_PRIO in ("off", "none", ""):
        return None
    if _COMPUTE_PRIO == "auto":
        return -1 if use_for(tokens, width) else None
    return int(_COMPUTE_PRIO)


@contextlib.contextmanager
def compute_stream(device: torch.device, tokens: int, width: Optional[int] = None):
    """Run the enclosed forward + backward on a stream of priority :func:`compute_priority`
    (ordered after, and joined back into, the caller's current stream); a no-op on CPU or when
    no priority applies."""
    prio = compute_priority(tokens, width) if device.type == "cuda" else None
    # not inside a hipGraph capture: a fork onto a stream of another priority there crashed
    # capture_end (segfault in tests/test_dropout_grad_gpu.py's graph test); replays run without it
    if prio is None or torch.cuda.is_current_stream_capturing():
        yield
        return
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _compute.get((idx, prio))
    if s is None:
        s = _compute[(idx, prio)] = torch.cuda.Stream(device=idx, priority=prio)
    cur = torch.cuda.current_stream(idx)
    s.wait_stream(cur)
    try:
        with torch.cuda.stream(s):
            yield
    finally:
        cur.wait_stream(s)


def run_wgrad(fn: Callable[[], None], *inputs: torch.Tensor) -> None:
    """Run ``fn`` (a weight-gradient accumulation reading ``inputs``) on the side stream."""
    if not inputs[0].is_cuda or not use_for(inputs[0].shape[0], min(t.shape[-1] for t in inputs)):
        fn()
        return
    dev = inputs[0].device
    s = _stream(dev)
    cur = torch.cuda.current_stream(dev)
    q = _inflight.setdefault(s.device.index, deque())
    while len(q) >= _LAG:  # the oldest weight gradient's inputs may now be reused by `cur`
        ev, _ = q.popleft()
        cur.wait_event(ev)
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        fn()
    ev = torch.cuda.Event()
    ev.record(s)
    q.append((ev, inputs))
    _pending.add(s.device.index)


def join() -> None:
    """The compute stream waits for every weight gradient issued so far (no host block)."""
    if not _pending:
        return
    for idx in list(_pending):
        torch.cuda.current_stream(idx).wait_stream(_side[idx])
        _inflight.get(idx, deque()).clear()  # inputs released only after the wait
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
