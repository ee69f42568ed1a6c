"""ZeRO-1: optimizer state sharded over the data-parallel ranks.

SURVEY §2.4 lists FSDP/ZeRO as absent from the reference (its only strategy is DDP,
``/root/reference/mingpt/trainer.py:71``) and as the optional next step after replicated DP.
This is that step, built on the same flat buffers as :class:`DataParallelEngine`:

* The :class:`~mingpt_distributed_amd.optim.FlatParamStore` is padded to ``world * 64``
  elements, so rank ``r`` owns the contiguous, 16-byte aligned range ``[r*S, (r+1)*S)``.
* **Gradients**: one ``reduce_scatter_tensor`` of the fp32 main-grad buffer at the step
  boundary leaves each rank the summed gradient of its own shard (``(N-1)/N`` of the buffer over
  the links, half of a ring all-reduce's traffic).  It is not overlapped with backward: a single
  large collective is the bandwidth-optimal shape for point-to-point xGMI rings, and the
  optimizer needs the whole shard anyway.
* **Optimizer**: the ``adamw.hip`` kernels run unchanged on the shard slices (chunk table
  relative to the shard).  The global grad norm is the all-reduced sum of per-shard sums of
  squares, so clipping matches the replicated optimizer exactly.  Adam moments are allocated
  for the shard only: ``8 * P / N`` bytes per rank instead of ``8 * P``.
* **Parameters**: ``all_gather_into_tensor`` of the bf16 compute shard (half the bytes of the
  fp32 master) rebuilds the full compute weights on every rank.  fp32 master weights outside
  the shard go stale; :meth:`ZeroAdamW.consolidate` (collective) gathers masters and moments
  before a snapshot, so checkpoints keep the replicated optimizer's format and load either way.
"""
from __future__ import annotations

import math
from typing import Optional, Set

import torch
import torch.distributed as dist

from ..optim import ALIGN, CHUNK, FlatParamStore, FusedAdamW
from .ddp import DataParallelEngine


class ZeroGradEngine(DataParallelEngine):
    """Gradient side of ZeRO-1: readiness bookkeeping as in DP, one reduce-scatter per step."""

    def __init__(self, store: FlatParamStore, process_group=None, broadcast: bool = True):
        super().__init__(store, process_group, bucket_mb=float(store.total * 4) / 2 ** 20 + 1,
                         broadcast=broadcast)
        assert store.total % (self.world * ALIGN) == 0, "store must be padded to world * ALIGN"
        self.rank = dist.get_rank(process_group)
        self.shard = store.total // self.world
        self.lo = self.rank * self.shard
        self.hi = self.lo + self.shard
        dev = store.device
        self.grad_shard = torch.zeros(self.shard, dtype=torch.float32, device=dev)
        self.param_stage = torch.empty(self.shard, dtype=store.flat.dtype, device=dev)
        # gloo with device tensors (the 2-ranks-on-one-card GPU tests): stage through the list
        # collectives gloo implements for CUDA; RCCL takes the *_tensor fast path
        self._gloo_dev = dev.type == "cuda" and dist.get_backend(process_group) == "gloo"

    def _launch_ready(self):
        return  # no per-bucket collectives: the reduce-scatter runs at the step boundary

    def finish(self):
        if self.world > 1 and self.sync_enabled:
            if self._gloo_dev:
                dist.all_reduce(self.store.grad, op=dist.ReduceOp.SUM, group=self.pg)
                self.grad_shard.copy_(self.store.grad[self.lo:self.hi])
            else:
                dist.reduce_scatter_tensor(self.grad_shard, self.store.grad, op=dist.ReduceOp.SUM,
                                           group=self.pg)
        for b in self.buckets:
            b.ready = 0
        self.done = [False] * len(self.done)
        self.uses = [0] * len(self.uses)

    def gather(self, full: torch.Tensor, shard_src: Optional[torch.Tensor] = None):
        """All-gather rank shards of ``full`` (in place; the local shard is staged first)."""
        src = full[self.lo:self.hi] if shard_src is None else shard_src
        stage = self.param_stage if src.dtype == self.param_stage.dtype else src.clone()
        if stage is self.param_stage:
            stage.copy_(src)
        self._all_gather(full, stage)

    def _all_gather(self, full: torch.Tensor, shard: torch.Tensor):
        if self._gloo_dev:
            dist.all_gather(list(full.chunk(self.world)), shard, group=self.pg)
        else:
            dist.all_gather_into_tensor(full, shard, group=self.pg)


class ZeroAdamW(FusedAdamW):
    """:class:`FusedAdamW` over this rank's shard of the flat buffers (see module docstring)."""

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
        lo, hi = engine.lo, engine.hi
        self.exp_avg = torch.zeros(hi - lo, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(hi - lo, dtype=torch.float32, device=dev)
        self.norm_buf = torch.zeros(2, dtype=torch.float32, device=dev)
        # per-parameter pieces inside the shard (shard-relative), then CHUNK-sized kernel chunks
        self.pieces = []
        for name, o, n in zip(store.names, store.offsets, store.numels):
            a, b = max(o, lo), min(o + n, hi)
            if a < b:
                self.pieces.append((a - lo, b - lo, self.wd_of[name]))
        starts, lens, wds = [], [], []
        for a, b, wd in self.pieces:
            for c in range(a, b, CHUNK):
                starts.append(c)
                lens.append(min(CHUNK, b - c))
                wds.append(wd)
        self.n_chunks = len(starts)
        self.c_start = torch.tensor(starts, dtype=torch.int64, device=dev)
        self.c_len = torch.tensor(lens, dtype=torch.int32, device=dev)
        self.c_wd = torch.tensor(wds, dtype=torch.float32, device=dev)
        self._full_state = None
        self.param_groups = [{"lr": lr, "betas": self.betas, "weight_decay": weight_decay, "eps": eps}]

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None):
        s, e = self.store, self.engine
        lr = self.param_groups[0]["lr"] if lr is None else lr
        self.step_count += 1
        self._full_state = None
        b1, b2 = self.betas
        master, flat, g = s.master[e.lo:e.hi], s.flat[e.lo:e.hi], e.grad_shard
        if s.device.type == "cuda":
            from ..ops._ext import ext

            C = ext()
            C.grad_sumsq(g, grad_scale, self.norm_buf)  # [0] = local sum of squares (unscaled)
            dist.all_reduce(self.norm_buf[:1], group=e.pg)
            torch.mul(self.norm_buf[:1].sqrt(), grad_scale, out=self.norm_buf[1:])
            if self.n_chunks:
                C.adamw_step(self.c_start, self.c_len, self.c_wd, master, flat, g, self.exp_avg,
                             self.exp_avg_sq, self.norm_buf, lr, b1, b2, self.eps, self.step_count,
                             grad_scale, float(self.grad_clip))
            e.gather(s.flat)
            return
        # CPU path (same math as FusedAdamW's, on the shard)
        gs = g * grad_scale
        self.norm_buf[0] = (gs * gs).sum()
        dist.all_reduce(self.norm_buf[:1], group=e.pg)
        self.norm_buf[1] = self.norm_buf[0].sqrt()
        if self.grad_clip > 0:
            coef = self.grad_clip / (self.norm_buf[1] + 1e-6)
            if coef < 1:
                gs = gs * coef
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        self.exp_avg.mul_(b1).add_(gs, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(gs, gs, value=1 - b2)
        for a, b, wd in self.pieces:
            if wd:
                master[a:b].mul_(1 - lr * wd)
            denom = (self.exp_avg_sq[a:b].sqrt() / math.sqrt(bc2)).add_(self.eps)
            master[a:b].addcdiv_(self.exp_avg[a:b], denom, value=-lr / bc1)
        if s.flat is not s.master:
            flat.copy_(master)
        e.gather(s.flat)

    # ------------------------------------------------------------------ state
    def consolidate(self):
        """Collective: gather fp32 masters and both moments onto every rank (before a snapshot)."""
        s, e = self.store, self.engine
        e.gather(s.master)
        m = torch.empty(s.total, dtype=torch.float32, device=s.device)
        v = torch.empty_like(m)
        e._all_gather(m, self.exp_avg)
        e._all_gather(v, self.exp_avg_sq)
        self._full_state = (m, v)

    def state_dict(self):
        if self._full_state is None:
            raise RuntimeError("ZeroAdamW.state_dict: call consolidate() on every rank first")
        m, v = self._full_state
        s = self.store
        st = {}
        for name, o, n, p in zip(s.names, s.offsets, s.numels, s.params):
            st[name] = {"exp_avg": m[o:o + n].view(p.shape).cpu().clone(),
                        "exp_avg_sq": v[o:o + n].view(p.shape).cpu().clone(),
                        "master": s.master[o:o + n].view(p.shape).cpu().clone()}
        return {"step": self.step_count, "state": st,
                "hparams": {"lr": self.param_groups[0]["lr"], "betas": list(self.betas), "eps": self.eps,
                            "weight_decay": self.weight_decay, "grad_clip": self.grad_clip}}

    def load_state_dict(self, sd):
        """Every rank loads the full (replicated-format) state and keeps its shard."""
        s, e = self.store, self.engine
        self.step_count = int(sd["step"])
        for name, o, n in zip(s.names, s.offsets, s.numels):
            ent = sd["state"].get(name)
            if ent is None:
                continue
            if "master" in ent:
                s.master[o:o + n].copy_(ent["master"].reshape(-1))
            a, b = max(o, e.lo), min(o + n, e.hi)
            if a < b:
                self.exp_avg[a - e.lo:b - e.lo].copy_(ent["exp_avg"].reshape(-1)[a - o:b - o])
                self.exp_avg_sq[a - e.lo:b - e.lo].copy_(ent["exp_avg_sq"].reshape(-1)[a - o:b - o])
        s.sync_params_from_master()
        self._full_state = None
