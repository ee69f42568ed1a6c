"""Native RCCL communicator for the data-parallel engines (``csrc/comm/rccl_comm.cpp``).

The reference's gradient traffic goes through c10d ``ProcessGroupNCCL`` inside DDP
(``/root/reference/mingpt/train.py:34``, ``trainer.py:71``).  With ``comm="rccl"`` (or
``MINGPT_COMM=rccl``) :class:`~.ddp.DataParallelEngine` and :class:`~.zero.ZeroGradEngine` drive
RCCL themselves instead:

* **Bootstrap** over the existing process group: rank 0's ``ncclGetUniqueId`` bytes are broadcast
  (``broadcast_object_list``), then every rank calls ``ncclCommInitRank`` on its GPU.  The RCCL is
  the one torch already loaded (``torch/lib/librccl.so``, soname ``librccl.so.1``), bound by
  ``dlopen(RTLD_NOLOAD)`` -- never a second RCCL from ``/opt/rocm``.
* **One comm stream** (highest HIP priority) per communicator.  A collective first makes the comm
  stream wait for everything the caller's current stream has enqueued (the bucket's producers:
  an event, no host sync), and returns a :class:`Work` whose ``wait()`` makes the current stream
  wait for the collective's completion event -- the same contract as c10d's
  ``async_op=True`` work on RCCL, without c10d's per-call bookkeeping, watchdog or work objects.
* Sums only (gradients); in-place all-reduce, reduce-scatter into the caller's own slice of the
  bucket, all-gather out of it, broadcast.

c10d stays the default: the native path is exercised on one GPU (a one-rank communicator,
``tests/test_comm_gpu.py``) and is **not yet verified at world > 1** (the pool's GPU boxes have
one GPU; ``tests/test_dp_gpu.py::test_gpu_nccl_two_gpus_match_single_process[rccl]`` covers it
on a multi-GPU node).  When an engine owns a native communicator, every collective of its step
goes through it (the ZeRO-1 grad-norm all-reduce included), so one step never mixes two
communicators' streams.
"""
from __future__ import annotations

import atexit
import os
import weakref
from typing import Optional

import torch
import torch.distributed as dist


def _torch_rccl_path() -> str:
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


def comm_backend_default() -> str:
    """``MINGPT_COMM``: ``c10d`` (default) or ``rccl`` (this module)."""
    v = os.environ.get("MINGPT_COMM", "c10d").lower()
    if v not in ("c10d", "rccl"):
        raise ValueError(f"MINGPT_COMM must be c10d or rccl, not {v!r}")
    return v


def _close_if_alive(ref):
    c = ref()
    if c is not None:
        c.close()


class Work:
    """One collective in flight: ``wait()`` orders the caller's current stream after it.  A Work
    dropped without ``wait()`` (an exception between launch and finish, an engine closed with
    buckets in flight) retires its ticket when collected, so the communicator's outstanding
    tickets do not grow for its lifetime."""

    __slots__ = ("_comm", "_ticket")

    def __init__(self, comm: "RcclCommunicator", ticket: int):
        self._comm, self._ticket = comm, ticket

    def wait(self):
        if self._ticket is not None:
            self._comm._C.comm_wait(self._comm.handle, self._ticket)
            self._ticket = None

    def is_completed(self) -> bool:
        """True once the collective has finished on the device (or was waited on / retired):
        a host-side query, no synchronisation (hang diagnostics)."""
        if self._ticket is None or not self._comm.handle:
            return True
        return self._comm._C.comm_query(self._comm.handle, self._ticket) != 0

    def retire(self):
        if self._ticket is not None and self._comm.handle:
            self._comm._C.comm_retire(self._comm.handle, self._ticket)
        self._ticket = None

    def __del__(self):
        try:
            self.retire()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class RcclCommunicator:
    """An RCCL communicator over the ranks of ``process_group`` on ``device`` (see module doc)."""

    def __init__(self, process_group=None, device: Optional[torch.device] = None):
        from ..ops._ext import ext

        if not dist.is_initialized():
            raise RuntimeError("RcclCommunicator: initialise torch.distributed first (bootstrap store)")
        device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("RcclCommunicator: a GPU device is required (RCCL)")
        self._C = ext()
        self.version = int(self._C.comm_load(_torch_rccl_path()))
        self.pg = process_group
        self.rank = dist.get_rank(process_group)
        self.world = dist.get_world_size(process_group)
        self.device = device
        box = [self._C.comm_unique_id() if self.rank == 0 else None]
        src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        dist.broadcast_object_list(box, src=src, group=process_group)
        with torch.cuda.device(device):
            self.handle = int(self._C.comm_create(box[0], self.world, self.rank, device.index))
        self.stream = torch.cuda.ExternalStream(int(self._C.comm_stream_ptr(self.handle)), device=device)
        # tear RCCL down before the interpreter (and torch's own atexit teardown of HIP / c10d):
        # atexit runs handlers last-registered first, and this one is registered after torch's.
        # Through a weak reference, so the handler does not keep a dropped communicator (and its
        # RCCL resources) alive until exit; __del__ closes it when it is collected
        atexit.register(_close_if_alive, weakref.ref(self))

    @property
    def version_str(self) -> str:
        v = self.version
        return f"{v // 10000}.{(v // 100) % 100}.{v % 100}"

    def _tensor(self, t: torch.Tensor) -> torch.Tensor:
        t.record_stream(self.stream)  # the comm stream uses it: keep the allocator from reusing it early
        return t

    def all_reduce(self, t: torch.Tensor) -> Work:
        """In-place sum over ranks (any dtype RCCL sums: fp32 / bf16 / fp16 / int64)."""
        return Work(self, int(self._C.comm_all_reduce(self.handle, self._tensor(t))))

    def reduce_scatter(self, inp: torch.Tensor, out: torch.Tensor) -> Work:
        """``out`` (numel = inp.numel() / world) <- this rank's slice of the sum of ``inp`` over
        ranks; ``out`` may be that slice of ``inp`` itself (in place)."""
        return Work(self, int(self._C.comm_reduce_scatter(self.handle, self._tensor(inp), self._tensor(out))))

    def all_gather(self, inp: torch.Tensor, out: torch.Tensor) -> Work:
        """``out`` (numel = world x inp.numel()) <- every rank's ``inp`` in rank order; ``inp``
        may be this rank's slice of ``out`` (in place)."""
        return Work(self, int(self._C.comm_all_gather(self.handle, self._tensor(inp), self._tensor(out))))

    def broadcast(self, t: torch.Tensor, src: int = 0) -> Work:
        return Work(self, int(self._C.comm_broadcast(self.handle, self._tensor(t), int(src))))

    def pending(self) -> int:
        return int(self._C.comm_pending(self.handle))

    def close(self):
        """Destroy the RCCL communicator (idempotent; its comm stream stays, see rccl_comm.cpp)."""
        if getattr(self, "handle", None):
            self._C.comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass
