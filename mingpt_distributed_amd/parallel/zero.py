"""ZeRO-1: optimizer state sharded over the data-parallel ranks, communication overlapped.

SURVEY §2.4 lists FSDP/ZeRO as absent from the reference (its only strategy is DDP,
``/root/reference/mingpt/trainer.py:71``) and as the optional next step after replicated DP.
This is that step, built on the same flat buffers and bucket layout as
:class:`DataParallelEngine`:

* **Layout.**  The :class:`~mingpt_distributed_amd.optim.FlatParamStore` is cut into buckets
  padded to ``world * 64`` elements; rank ``r`` owns the ``r``-th equal slice of EVERY bucket
  (interleaved shards), so each bucket's collective is one equal-split reduce-scatter.
* **Gradients.**  A bucket's ``reduce_scatter_tensor`` launches from inside backward the moment
  its last gradient lands (same readiness protocol as DP), on RCCL **in place**: the output is
  the rank's own slice of the input (``out == in + rank * count``), so no gradient shard buffer
  exists.  ``(N-1)/N`` of the bucket crosses the links: half a ring all-reduce.  With
  ``reduce_dtype=bf16`` the bucket is converted into a bf16 comm buffer first and the optimizer
  reads bf16 gradients.
* **Optimizer.**  The ``adamw.hip`` kernels run on the rank's pieces through a chunk table whose
  moment offsets are packed (``moment_start``): Adam moments exist for the shard only,
  ``8 * P / N`` bytes per rank.  The global grad norm is the all-reduced sum of per-shard sums of
  squares, so clipping equals the replicated optimizer's.
* **Parameters.**  After the update each bucket's bf16 compute weights are all-gathered in place
  (input = own slice of the output), asynchronously.  The next forward waits per bucket, right
  before the first kernel that reads one of its weights (``ops/grads.before_use``): the gather of
  later layers overlaps the forward of earlier ones.  Forwards that do not go through the fused
  GPU ops (CPU path, ``no_grad`` inference, models other than this package's GPT) wait for
  everything up front in a forward pre-hook; ``generate`` (whose KV-cache decode calls the
  kernels directly, never ``model.forward``) waits through ``before_use`` on every parameter.
* **Snapshots.**  The fp32 master is replicated in memory, but only the rank's pieces are
  current: :meth:`ZeroAdamW.consolidate` (collective) all-gathers masters in place (no extra
  memory) and streams each bucket's moment slices to rank 0, which copies them to host memory.
  No rank ever holds the full moments on the device; rank 0's host copy is dropped as soon as
  :meth:`state_dict` has read it.
* ``world == 1`` runs the same code with the collectives skipped (shard = everything).
"""
from __future__ import annotations

import math
from typing import List, Optional, Set

import torch
import torch.distributed as dist

from ..ops import streams
from ..optim import FlatParamStore, FusedAdamW, make_chunk_table
from .ddp import DataParallelEngine, _Bucket


class ZeroGradEngine(DataParallelEngine):
    """Gradient and parameter side of ZeRO-1 (see module docstring)."""

    collective_kind = "reduce_scatter + all_gather (bf16 params)"

    def __init__(self, store: FlatParamStore, process_group=None, broadcast: bool = True,
                 reduce_dtype: Optional[torch.dtype] = None, model: Optional[torch.nn.Module] = None,
                 comm_at_world1: bool = False, comm: Optional[str] = None, native=None):
        super().__init__(store, process_group, reduce_dtype=reduce_dtype, broadcast=broadcast,
                         comm_at_world1=comm_at_world1, comm=comm, native=native)
        multi = self.active
        self.rank = dist.get_rank(process_group) if multi else 0
        for s, e, _ in store.buckets:
            if (e - s) % (self.world * 64):
                raise ValueError("ZeRO-1 needs every bucket padded to world * 64 elements")
        # this rank's slice of every bucket: (bucket start, end, own lo, own hi)
        self.own = []
        for b in self.buckets:
            sh = (b.end - b.start) // self.world
            lo = b.start + self.rank * sh
            self.own.append((lo, lo + sh))
        self.shard_numel = sum(hi - lo for lo, hi in self.own)
        self.gather_work: List[Optional[object]] = [None] * len(self.buckets)
        # gloo (CPU tests, and two ranks sharing one GPU in tests/test_dp_gpu.py) runs the same
        # in-place reduce_scatter_tensor / all_gather_into_tensor calls as RCCL (torch >= 2.6 has
        # both on gloo, host and device tensors); only consolidate()'s gather needs host tensors
        self._gloo = multi and dist.get_backend(process_group) == "gloo"
        self._hook_handle = None
        # Per-bucket waits are only sound when every weight read of a grad-enabled GPU forward
        # goes through a fused op that calls ``ops.grads.before_use`` first: the contract holds
        # for this package's GPT.forward (ops/fused.py) and is not assumed for anything else (a
        # subclass overriding forward, custom heads, user modules): those wait for everything.
        self._fused_forward = False
        if model is not None:
            from ..models.gpt import GPT

            self._fused_forward = isinstance(model, GPT) and type(model).forward is GPT.forward
        if multi and model is not None:
            self._hook_handle = model.register_forward_pre_hook(self._forward_pre_hook)

    # ------------------------------------------------------------------ gradients
    def _issue(self, b: _Bucket, wire: Optional[torch.Tensor] = None):
        wire = self._wire(b) if wire is None else wire
        bi = self.buckets.index(b)
        lo, hi = self.own[bi]
        out = wire[lo - b.start:hi - b.start]
        if self.native is not None:
            return self.native.reduce_scatter(wire, out)
        return dist.reduce_scatter_tensor(out, wire, op=dist.ReduceOp.SUM, group=self.pg,
                                          async_op=True)

    def finish(self):
        self.wait_gathers()  # weights no forward read this step are still owed to the optimizer
        super().finish()

    def bus_bytes(self, b: _Bucket) -> float:
        """Reduce-scatter: (N-1)/N x bucket bytes per rank."""
        esz = 2 if self.reduce_dtype == torch.bfloat16 else 4
        return (self.world - 1) / self.world * (b.end - b.start) * esz

    def relayout_order(self):
        self.observed = None  # moments are sharded by layout position: keep the layout
        return None

    # ------------------------------------------------------------------ parameters
    def gather_params(self):
        """Launch the in-place all-gather of every bucket's bf16 compute weights (async)."""
        if not self.active:
            return
        flat = self.store.flat
        for bi, b in enumerate(self.buckets):
            lo, hi = self.own[bi]
            full = flat[b.start:b.end]
            if self.native is not None:
                self.gather_work[bi] = self.native.all_gather(flat[lo:hi], full)
            else:
                self.gather_work[bi] = dist.all_gather_into_tensor(full, flat[lo:hi], group=self.pg,
                                                                   async_op=True)

    def before_use(self, p):
        bi = self.bucket_of[self.store.index[id(p)]]
        w = self.gather_work[bi]
        if w is not None:
            w.wait()  # stream-ordered on RCCL: the compute stream waits, the host does not
            self.gather_work[bi] = None

    def wait_gathers(self):
        for bi, w in enumerate(self.gather_work):
            if w is not None:
                w.wait()
                self.gather_work[bi] = None

    def _forward_pre_hook(self, module, args):
        idx = args[0] if args else None
        if not (self._fused_forward and isinstance(idx, torch.Tensor) and idx.is_cuda
                and torch.is_grad_enabled()):
            self.wait_gathers()

    def all_gather_inplace(self, buf: torch.Tensor):
        """Synchronously all-gather every bucket of a full-size flat buffer (e.g. fp32 masters)."""
        if not self.active:
            return
        for bi, b in enumerate(self.buckets):
            lo, hi = self.own[bi]
            full = buf[b.start:b.end]
            if self.native is not None:
                self.native.all_gather(buf[lo:hi], full).wait()
            else:
                dist.all_gather_into_tensor(full, buf[lo:hi], group=self.pg)

    def close(self):
        if self._hook_handle is not None:
            self._hook_handle.remove()
            self._hook_handle = None
        super().close()


class ZeroAdamW(FusedAdamW):
    """:class:`FusedAdamW` over this rank's pieces of the flat buffers (see module docstring)."""

    def __init__(self, store: FlatParamStore, engine: ZeroGradEngine, lr: float = 3e-4,
                 betas=(0.9, 0.95), eps: float = 1e-8, weight_decay: float = 0.1,
                 decay_names: Optional[Set[str]] = None, grad_clip: float = 0.0):
        self.store, self.engine = store, engine
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.grad_clip = grad_clip
        if decay_names is None:
            decay_names = {n for n, p in zip(store.names, store.params) if p.dim() >= 2}
        self.decay_names = set(decay_names)
        self.wd_of = {n: (weight_decay if n in self.decay_names else 0.0) for n in store.names}
        self.step_count = 0
        dev = store.device
        # packed moment offset of every bucket's own slice
        self.moff, off = [], 0
        for lo, hi in engine.own:
            self.moff.append(off)
            off += hi - lo
        self.exp_avg = torch.zeros(off, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(off, dtype=torch.float32, device=dev)
        self.norm_buf = torch.zeros(2, dtype=torch.float32, device=dev)
        # (global start, end, wd, packed moment start) of every parameter piece this rank owns
        self.pieces = []
        for (lo, hi), mo in zip(engine.own, self.moff):
            for a, b, wd in store.pieces(self.wd_of, lo, hi):
                self.pieces.append((a, b, wd, mo + (a - lo)))
        self.table = make_chunk_table(self.pieces, dev, store.total, off)
        self.n_chunks = int(self.table.len.numel())
        self._host_state = None
        self.param_groups = [{"lr": lr, "betas": self.betas, "weight_decay": weight_decay, "eps": eps}]

    @property
    def grad_buffer(self) -> torch.Tensor:
        return self.engine.grad_buffer

    @grad_buffer.setter
    def grad_buffer(self, _v):  # the engine owns it
        pass

    def _all_reduce_sumsq(self):
        """Global squared grad norm = sum of the shards' sums.  Through the engine's native
        communicator when it has one, so the step's collectives (reduce-scatters, this, the
        parameter all-gathers) all run in order on ONE comm stream."""
        if self.engine.active:
            if self.engine.native is not None:
                self.engine.native.all_reduce(self.norm_buf[:1]).wait()
            else:
                dist.all_reduce(self.norm_buf[:1], group=self.engine.pg)

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None):
        streams.join()  # weight gradients still on the side stream (ops/streams.py)
        s, e = self.store, self.engine
        lr = self.param_groups[0]["lr"] if lr is None else lr
        self.step_count += 1
        self._host_state = None
        b1, b2 = self.betas
        g = self.grad_buffer
        if s.device.type == "cuda":
            from ..ops._ext import ext

            C = ext()
            t = self.table
            C.grad_sumsq_chunks(t.start, t.len, g, grad_scale, self.norm_buf, t.end)
            self._all_reduce_sumsq()
            torch.mul(self.norm_buf[:1].sqrt(), grad_scale, out=self.norm_buf[1:])
            C.adamw_step(t.start, t.len, t.wd, t.mstart, s.master, s.flat, g,
                         self.exp_avg, self.exp_avg_sq, self.norm_buf, lr, b1, b2, self.eps,
                         self.step_count, grad_scale, float(self.grad_clip), t.end, t.mend)
            e.gather_params()
            return
        # CPU path (same math as FusedAdamW's, on the owned pieces)
        sq = torch.zeros((), dtype=torch.float32)
        for a, b, _, _ in self.pieces:
            ga = g[a:b].float() * grad_scale
            sq += (ga * ga).sum()
        self.norm_buf[0] = sq
        self._all_reduce_sumsq()
        self.norm_buf[1] = self.norm_buf[0].sqrt()
        coef = 1.0
        if self.grad_clip > 0:
            c = self.grad_clip / (self.norm_buf[1].item() + 1e-6)
            coef = min(1.0, c)
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        for a, b, wd, ma in self.pieces:
            gs = g[a:b].float() * (grad_scale * coef)
            m = self.exp_avg[ma:ma + b - a]
            v = self.exp_avg_sq[ma:ma + b - a]
            m.mul_(b1).add_(gs, alpha=1 - b1)
            v.mul_(b2).addcmul_(gs, gs, value=1 - b2)
            if wd:
                s.master[a:b].mul_(1 - lr * wd)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            s.master[a:b].addcdiv_(m, denom, value=-lr / bc1)
            if s.flat is not s.master:
                s.flat[a:b].copy_(s.master[a:b])
        e.gather_params()
        e.wait_gathers()  # CPU: the next forward reads the weights directly

    # ------------------------------------------------------------------ state
    def consolidate(self):
        """Collective.  Every rank: fp32 masters all-gathered in place (no extra memory).  Rank 0:
        the full Adam moments assembled in HOST memory, one bucket slice at a time (no rank ever
        holds the full moments on the device)."""
        s, e = self.store, self.engine
        e.wait_gathers()
        e.all_gather_inplace(s.master)
        is0 = e.rank == 0
        host = None
        if is0:
            host = (torch.zeros(s.total, dtype=torch.float32), torch.zeros(s.total, dtype=torch.float32))
        for bi, b in enumerate(e.buckets):
            lo, hi = e.own[bi]
            sh = hi - lo
            mo = self.moff[bi]
            for k, buf in enumerate((self.exp_avg, self.exp_avg_sq)):
                piece = buf[mo:mo + sh]
                if not e.active:
                    host[k][b.start:b.end].copy_(piece)
                    continue
                if e._gloo:
                    piece = piece.cpu()  # gloo gathers host tensors only
                parts = [torch.empty_like(piece) for _ in range(e.world)] if is0 else None
                dist.gather(piece, parts, dst=0, group=e.pg)
                if is0:
                    host[k][b.start:b.end].copy_(torch.cat(parts))
        self._host_state = host

    def state_dict(self):
        """Replicated-format optimizer state (loads into :class:`FusedAdamW` too).  Needs
        :meth:`consolidate` first; only rank 0 holds the consolidated moments."""
        if self._host_state is None:
            raise RuntimeError("ZeroAdamW.state_dict: call consolidate() on every rank first "
                               "(the full state is assembled on rank 0 only)")
        m, v = self._host_state
        self._host_state = None  # do not keep a host copy of the full moments around
        s = self.store
        st = {}
        for name, o, n, p in zip(s.names, s.offsets, s.numels, s.params):
            st[name] = {"exp_avg": m[o:o + n].view(p.shape).clone(),
                        "exp_avg_sq": v[o:o + n].view(p.shape).clone(),
                        "master": s.master[o:o + n].view(p.shape).cpu().clone()}
        return {"step": self.step_count, "state": st,
                "hparams": {"lr": self.param_groups[0]["lr"], "betas": list(self.betas), "eps": self.eps,
                            "weight_decay": self.weight_decay, "grad_clip": self.grad_clip}}

    def load_state_dict(self, sd):
        """Every rank loads the full (replicated-format) state and keeps its pieces."""
        s = self.store
        self.step_count = int(sd["step"])
        for name, o, n in zip(s.names, s.offsets, s.numels):
            ent = sd["state"].get(name)
            if ent is not None and "master" in ent:
                s.master[o:o + n].copy_(ent["master"].reshape(-1))
        for a, b, _, ma in self.pieces:
            for name, o, n in zip(s.names, s.offsets, s.numels):
                if o <= a and b <= o + n:
                    ent = sd["state"].get(name)
                    if ent is not None:
                        self.exp_avg[ma:ma + b - a].copy_(ent["exp_avg"].reshape(-1)[a - o:b - o])
                        self.exp_avg_sq[ma:ma + b - a].copy_(ent["exp_avg_sq"].reshape(-1)[a - o:b - o])
                    break
        s.sync_params_from_master()
        self._host_state = None
