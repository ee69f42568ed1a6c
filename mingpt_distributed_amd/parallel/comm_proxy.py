"""One-GPU proxy for the gradient all-reduces of an N-GPU data-parallel step.

At N > 1 every bucket's all-reduce (``ddp.py`` ``_launch``, DDP's overlapped bucket reduction in
``/root/reference/mingpt/trainer.py:71``) runs as RCCL kernels on their own stream while backward
keeps the compute stream busy.  The step's GEMMs (``gemm.hip`` W4: all 160 KiB of LDS and the
whole register file of a CU per workgroup) leave no room beside them on a CU, so a collective's
workgroups get CUs only as GEMM workgroups retire.  Whether that makes the collectives queue
behind backward -- or slows backward by holding CUs -- is measurable on one GPU: this module
stands in for the collective with ``comm_proxy.hip``, a kernel on ``channels`` workgroups that
moves the bucket's bytes x 2 (N - 1) / N and is paced to a bus bandwidth, so it lasts as long as
the ring all-reduce would and holds as many CUs.

``DataParallelEngine(comm="proxy")`` (one-rank group, ``comm_at_world1``) issues it at every
bucket-ready point on the same stream hand-off as the real collective; gradients are left as
they are (the proxy writes a scratch buffer), so the step's arithmetic is the one-GPU step's.
``bench/comm_proxy.py`` reports each proxy's launch-to-completion time inside the step (from the
moment its bucket was ready on the device) against its isolated time, and the step slowdown.
Environment: ``MINGPT_PROXY_RANKS`` (N, default 8; 1 = a null proxy that launches nothing, to
separate the data-parallel plumbing from the CU sharing), ``MINGPT_PROXY_CHANNELS`` (workgroups,
default 32), ``MINGPT_PROXY_GBPS`` (bus bandwidth, default 300; 0 = unpaced).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch


class _ProxyWork:
    """Work handle with the stream-ordered wait contract of c10d / the native communicator."""

    __slots__ = ("end",)

    def __init__(self, end: torch.cuda.Event):
        self.end = end

    def wait(self):
        torch.cuda.current_stream().wait_event(self.end)

    def is_completed(self) -> bool:
        return self.end.query()


class CommProxy:
    def __init__(self, device: torch.device, ranks: Optional[int] = None, channels: Optional[int] = None,
                 gbps: Optional[float] = None):
        if device.type != "cuda":
            raise RuntimeError("comm='proxy' models GPU collectives; it needs GPU parameters")
        env = os.environ.get
        self.ranks = int(ranks if ranks is not None else env("MINGPT_PROXY_RANKS", "8"))
        self.channels = int(channels if channels is not None else env("MINGPT_PROXY_CHANNELS", "32"))
        self.gbps = float(gbps if gbps is not None else env("MINGPT_PROXY_GBPS", "300"))
        # ranks 1: a null proxy (nothing moved, no kernel): the data-parallel plumbing alone
        if self.ranks < 1 or not 0 < self.channels <= 1024 or self.gbps < 0:
            raise ValueError(f"comm proxy: ranks {self.ranks} (>= 1), channels {self.channels}, gbps {self.gbps}")
        self.device = device
        self.stream = torch.cuda.Stream(device=device)  # RCCL runs on a stream of its own
        self._scratch: Optional[torch.Tensor] = None
        self.record = False
        self.records: List[Tuple[int, torch.cuda.Event, torch.cuda.Event]] = []
        from ..ops._ext import ext

        self._C = ext()

    @property
    def factor(self) -> float:
        """Bytes moved per bucket byte: ring all-reduce, 2 (N - 1) / N."""
        return 2.0 * (self.ranks - 1) / self.ranks

    def all_reduce(self, wire: torch.Tensor) -> _ProxyWork:
        nbytes = wire.numel() * wire.element_size()
        if self._scratch is None or self._scratch.numel() < nbytes:
            self._scratch = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        ready, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.stream):
            ready.record()  # reached once the bucket's producers are done: the ready point
            self._C.comm_proxy(wire, self._scratch, self.factor, self.channels, self.gbps)
            end.record()
        wire.record_stream(self.stream)
        if self.record:
            self.records.append((nbytes, ready, end))
        return _ProxyWork(end)

    def take_records(self) -> List[Tuple[int, float]]:
        """(bucket bytes, ready-to-completion ms) of every proxy recorded since the last call."""
        out = []
        for nbytes, ready, end in self.records:
            end.synchronize()
            out.append((nbytes, ready.elapsed_time(end)))
        self.records = []
        return out

    def model_ms(self, nbytes: int) -> Optional[float]:
        """The paced duration of one proxy on ``nbytes`` (None when unpaced)."""
        return None if self.gbps <= 0 else self.factor * nbytes / (self.gbps * 1e9) * 1e3
