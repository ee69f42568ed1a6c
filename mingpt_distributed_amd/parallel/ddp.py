"""Data-parallel engine: bucketed gradient all-reduce over RCCL, overlapped with backward.

Replaces ``torch.nn.parallel.DistributedDataParallel`` as used by the reference
(``/root/reference/mingpt/trainer.py:71``; behaviour surveyed in SURVEY §2.7 C3-C5), designed
for one node of 8 MI355X on a point-to-point xGMI mesh:

* **Zero-copy buckets.**  Gradients live in the flat fp32 buffer of :class:`FlatParamStore`
  (``p.main_grad`` views) in backward-completion order, and the store cuts that buffer into
  buckets (``store.buckets``), so a bucket is a contiguous slice: no gradient->bucket copy and
  no copy back (DDP's K19 reducer copies).
* **Readiness by use counts.**  The fused GPU ops report each parameter use in forward and each
  gradient accumulation in backward (``ops/grads.py``); on the CPU path a
  ``post_accumulate_grad`` hook folds ``p.grad`` into ``main_grad``.  A bucket launches the
  moment its last gradient lands; buckets launch strictly in order so every rank issues the same
  collective sequence.
* **Overlap.**  ``dist.all_reduce(async_op=True)`` on the ``nccl`` (RCCL) backend runs on the
  process group's own HIP stream, ordered after the compute-stream kernels that produced the
  bucket, while backward keeps issuing kernels on the compute stream.  ``finish()`` makes the
  compute stream wait on the outstanding collectives (no host block) before the optimizer.
* **bf16 on the wire** (``reduce_dtype=torch.bfloat16``): a bucket is converted into a
  persistent bf16 comm buffer by one kernel the moment it is ready, reduced there in place, and
  the optimizer reads the reduced bf16 gradients directly (``FusedAdamW.grad_buffer``): half the
  link bytes, no per-step allocation and no copy back to fp32.
* **Bucket order from the observed backward.**  The first synchronised backward records the
  order in which parameters became ready; if it differs from the layout (a model whose
  registration order is not its reverse use order), :meth:`relayout_order` returns it and the
  step engine rebuilds the store in that order after the first optimizer step, as DDP rebuilds
  its buckets after iteration 1.
* **Sizing.**  Default 32 MiB fp32 buckets: big enough that each ring all-reduce is bandwidth-
  rather than latency-bound on xGMI (7 links x ~153 GB/s per GPU), small enough that the first
  bucket launches early in backward.  The tied ``wte`` (its last use is the embedding backward,
  the final kernel of backward) sits alone in the last bucket, so what is exposed after
  backward is exactly that one reduction.
* The average over ranks (1/world) is folded into the optimizer's grad scale; the constant
  causal mask is never broadcast (there is no mask buffer; fixes D30).
* **Communicator**: c10d's RCCL process group by default, or (``comm="rccl"`` /
  ``MINGPT_COMM=rccl``) the engine's own RCCL communicator and comm stream
  (:mod:`.comm`, ``csrc/comm/rccl_comm.cpp``) with the same stream-ordered wait contract.
  ``comm="proxy"`` (one-rank group only): :mod:`.comm_proxy`'s one-GPU stand-in for an N-rank
  all-reduce's CU occupancy and duration, for measuring comm/compute CU sharing on one GPU.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import streams
from ..optim import FlatParamStore


class _Bucket:
    __slots__ = ("start", "end", "params", "ready", "work")

    def __init__(self, start, end, params):
        self.start, self.end, self.params = start, end, params
        self.ready = 0
        self.work = None


def _to_bf16(src: torch.Tensor, dst: torch.Tensor):
    if src.is_cuda:
        from ..ops._ext import ext

        ext().f32_to_bf16(src, dst)
    else:
        dst.copy_(src)


class DataParallelEngine:
    def __init__(self, store: FlatParamStore, process_group=None, bucket_mb: float = 32.0,
                 reduce_dtype: Optional[torch.dtype] = None, broadcast: bool = True,
                 comm_at_world1: bool = False, comm: Optional[str] = None, native=None, proxy=None):
        """``comm_at_world1`` runs the collective path even in a one-rank process group (tests
        of the RCCL calls on a one-GPU box); otherwise one rank means no communication.
        ``comm``: ``"c10d"`` or ``"rccl"`` (native communicator; default ``MINGPT_COMM``), GPU
        stores only; ``native``: an existing :class:`~.comm.RcclCommunicator` to reuse (rebuilt
        engines after a bucket relayout); ``proxy``: likewise an existing comm proxy."""
        self.store = store
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.active = self.world > 1 or (comm_at_world1 and dist.is_initialized())
        if reduce_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError("reduce_dtype must be None/float32 or bfloat16")
        self.reduce_dtype = None if reduce_dtype == torch.float32 else reduce_dtype
        self.bucket_mb = bucket_mb
        self.sync_enabled = True
        self.buckets: List[_Bucket] = [_Bucket(s, e, ps) for s, e, ps in store.buckets]
        self.bucket_of = {}
        for bi, b in enumerate(self.buckets):
            for i in b.params:
                self.bucket_of[i] = bi
        self.uses = [0] * len(store.params)
        self.done = [False] * len(store.params)
        self.next_launch = 0
        self._hooks = []
        # (bucket index, elements, work) of the latest synchronised step, kept after finish() for
        # hang diagnostics (bench.py's watchdog names the first bucket whose collective has not
        # completed); replaced at the next step's first launch
        self.inflight: List[tuple] = []
        self.comm = None  # bf16 reduce buffer (same layout as store.grad)
        self.observed: Optional[List[int]] = None  # ready order of the first synchronised backward
        self._recording: Optional[List[int]] = []
        from .comm import RcclCommunicator, comm_backend_default

        self.comm_backend = comm or comm_backend_default()
        self.native = None
        self.proxy = None
        if self.active and self.comm_backend == "proxy":
            if self.world != 1:
                raise RuntimeError("comm='proxy' stands in for the ranks of a one-rank group only")
            from .comm_proxy import CommProxy

            self.proxy = proxy if proxy is not None else CommProxy(store.device)
        elif self.active and self.comm_backend == "rccl":
            if store.device.type != "cuda":
                raise RuntimeError("comm='rccl' needs GPU parameters (RCCL); use c10d for CPU runs")
            self.native = native if native is not None else RcclCommunicator(process_group, store.device)
        if self.active:
            if self.reduce_dtype is not None:
                self.comm = torch.empty(store.total, dtype=self.reduce_dtype, device=store.device)
            for p in store.params:
                p._mg_engine = self
                self._hooks.append(p.register_post_accumulate_grad_hook(self._cpu_grad_hook))
            if broadcast:
                self.broadcast_params()

    @staticmethod
    def bucket_numel(bucket_mb: float) -> int:
        return max(1, int(bucket_mb * 1024 * 1024 / 4))

    @property
    def grad_buffer(self) -> torch.Tensor:
        """The buffer holding the reduced gradients after :meth:`finish`."""
        return self.comm if self.comm is not None else self.store.grad

    # ------------------------------------------------------------------ setup
    def broadcast_params(self, src: int = 0):
        """Make the weights of GROUP rank ``src`` of the engine's process group authoritative
        (DDP ctor broadcast, C3).  Both backends read ``src`` as a group rank: the native
        communicator's ranks are the group's, and c10d's ``broadcast`` takes a global rank, so
        it is converted (the two agree on the default group, and differ on a sub-group)."""
        if self.native is not None:
            self.native.broadcast(self.store.master, src).wait()
        else:
            gsrc = dist.get_global_rank(self.pg, src) if self.pg is not None else src
            dist.broadcast(self.store.master, gsrc, group=self.pg)
        self.store.sync_params_from_master()

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world

    # ------------------------------------------------------------------ readiness protocol
    def before_use(self, p):
        """Called before a forward reads ``p`` (ZeRO-1 waits for its parameter gather here)."""

    def note_use(self, p):
        self.uses[self.store.index[id(p)]] += 1

    def grad_done(self, p):
        i = self.store.index[id(p)]
        self.uses[i] -= 1
        if self.uses[i] <= 0:
            self._param_ready(i)

    def _cpu_grad_hook(self, p):
        if p.grad is not None:
            p.main_grad.add_(p.grad.to(p.main_grad.dtype))
            p.grad = None
        self._param_ready(self.store.index[id(p)])

    def _param_ready(self, i):
        if self.done[i]:
            return
        self.done[i] = True
        if self.sync_enabled and self._recording is not None:
            self._recording.append(i)
        b = self.buckets[self.bucket_of[i]]
        b.ready += 1
        if self.sync_enabled:
            self._launch_ready()

    def _launch_ready(self):
        while self.next_launch < len(self.buckets):
            b = self.buckets[self.next_launch]
            if b.ready < len(b.params):
                return
            self._launch(b)
            self.next_launch += 1

    def _wire(self, b: _Bucket) -> torch.Tensor:
        """The bucket's slice in the dtype it travels in (converted now if bf16)."""
        view = self.store.grad[b.start:b.end]
        if self.comm is None:
            return view
        out = self.comm[b.start:b.end]
        _to_bf16(view, out)
        return out

    def _launch(self, b: _Bucket):
        if self.next_launch == 0:
            self.inflight = []
        # after the bucket's weight gradients, which may still run on the side stream
        with streams.collective_stream(self.store.device):
            b.work = self._issue(b)
        self.inflight.append((self.next_launch, b.end - b.start, b.work))

    def _issue(self, b: _Bucket, wire: Optional[torch.Tensor] = None):
        """Start the bucket's collective on ``wire`` (default: the bucket's slice in the wire
        dtype, converted now); returns its work handle."""
        wire = self._wire(b) if wire is None else wire
        if self.proxy is not None:
            return self.proxy.all_reduce(wire)
        if self.native is not None:
            return self.native.all_reduce(wire)
        return dist.all_reduce(wire, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def time_collectives(self, reps: int = 5) -> List[float]:
        """Isolated time of every bucket's collective, in launch order (ms per collective, mean
        of ``reps`` back-to-back calls after a barrier): device time between events on the
        compute stream on GPUs, host wall time on CPU.  Diagnostics for bench.py, run AFTER the
        timed steps: it zeroes the wire buffer (sums of zeros stay finite) and leaves no result
        anyone reads."""
        if not self.active:
            return []
        wire_buf = self.comm if self.comm is not None else self.store.grad
        wire_buf.zero_()
        cuda = wire_buf.is_cuda
        out = []
        for b in self.buckets:
            wire = wire_buf[b.start:b.end]
            self._issue(b, wire).wait()  # warm (first use of this size)
            dist.barrier(group=self.pg)
            if cuda:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
                for _ in range(reps):
                    self._issue(b, wire).wait()
                ev[1].record()
                ev[1].synchronize()
                out.append(ev[0].elapsed_time(ev[1]) / reps)
            else:
                import time

                t0 = time.perf_counter()
                for _ in range(reps):
                    self._issue(b, wire).wait()
                out.append((time.perf_counter() - t0) * 1e3 / reps)
        return out

    def bus_bytes(self, b: _Bucket) -> float:
        """Bytes each rank moves over its links for the bucket's collective (ring accounting,
        the "bus bandwidth" convention): all-reduce 2 (N-1)/N x bucket bytes."""
        esz = 2 if self.reduce_dtype == torch.bfloat16 else 4
        return 2.0 * (self.world - 1) / self.world * (b.end - b.start) * esz

    def incomplete_collectives(self) -> List[tuple]:
        """(bucket index, elements) of the latest step's collectives that have not completed on
        the device -- a host-side query, safe from a watchdog thread (diagnostics only)."""
        out = []
        for k, n, w in list(self.inflight):
            try:
                done = w.is_completed()
            except Exception:  # noqa: BLE001 -- diagnostics only
                done = False
            if not done:
                out.append((k, n))
        return out

    # ------------------------------------------------------------------ step boundary
    def _wait_all(self):
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()  # stream-ordered: the compute stream waits, the host does not
            b.work = None
            b.ready = 0

    def finish(self):
        """Launch what is left (parameters unused this step), wait, and reset for the next step."""
        streams.join()
        if not self.active:
            return
        if self.sync_enabled:
            for i in range(len(self.done)):
                if not self.done[i]:
                    self.done[i] = True
                    self.buckets[self.bucket_of[i]].ready += 1
            self._launch_ready()
            self._wait_all()
            self.next_launch = 0
            if self._recording is not None:
                seen = set(self._recording)
                self.observed = self._recording + [i for i in range(len(self.done)) if i not in seen]
                self._recording = None
        else:
            # no_sync micro-step: keep counts clear for the next micro-step
            for b in self.buckets:
                b.ready = 0
        self.done = [False] * len(self.done)
        self.uses = [0] * len(self.uses)

    def relayout_order(self) -> Optional[List[str]]:
        """Parameter names in observed gradient-ready order if that differs from the layout
        (buckets would wait on late gradients), else None.  Consumed once.

        Collective (once, at the step after the first synchronised backward, which is the same
        step on every rank) when the engine communicates: each rank observes its OWN order, and
        ranks whose bucket boundaries differed would issue collectives of different sizes (hang
        or silent corruption), so rank 0's decision is broadcast and every rank adopts it."""
        obs, self.observed = self.observed, None
        if obs is None:
            return None
        order = None
        seq = [self.bucket_of[i] for i in obs]
        # buckets complete in launch order: order inside a bucket is irrelevant
        if not all(a <= b for a, b in zip(seq, seq[1:])):
            order = [self.store.names[i] for i in obs]
        if self.active and self.world > 1:
            box = [order]
            src = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
            dist.broadcast_object_list(box, src=src, group=self.pg)
            order = box[0]
            if order is not None and sorted(order) != sorted(self.store.names):
                raise RuntimeError("relayout_order: rank 0's parameter order names other parameters")
        return order

    def comm_plan(self) -> dict:
        """What one synchronised step puts on the wire (bench/diagnostics): bucket count, bytes
        of every bucket in launch order (wire dtype), the collective kind."""
        esz = 2 if self.reduce_dtype == torch.bfloat16 else 4
        return {"n_buckets": len(self.buckets),
                "bucket_bytes": [(b.end - b.start) * esz for b in self.buckets],
                "wire_dtype": "bf16" if esz == 2 else "fp32",
                "collective": self.collective_kind,
                "comm_backend": "proxy" if self.proxy is not None else
                "rccl-native" if self.native is not None else "c10d"}

    collective_kind = "all_reduce"

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation: skip communication for the enclosed micro-steps."""
        prev = self.sync_enabled
        self.sync_enabled = False
        try:
            yield
        finally:
            self.sync_enabled = prev

    def close(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for b in self.buckets:  # an unwaited native Work releases its ticket (no stream wait)
            if b.work is not None and hasattr(b.work, "retire"):
                b.work.retire()
            b.work = None
        self.inflight = []
        for p in self.store.params:
            if getattr(p, "_mg_engine", None) is self:
                del p._mg_engine
