"""Optimizer layer: the reference's decay grouping, flat parameter storage, fused AdamW.

* :func:`param_groups` / :func:`create_optimizer` reproduce the reference's decay rules
  (``/root/reference/mingpt/model.py:62-122``): Linear weights decay; biases, LayerNorm and
  Embedding weights do not; the sets must be disjoint and complete.  ``create_optimizer`` returns
  a plain ``torch.optim.AdamW`` (API parity; the trainer converts it to :class:`FusedAdamW`).
* :class:`FlatParamStore` re-homes every parameter into ONE flat buffer per role, sized for HBM
  (not for copies): bf16 compute params, fp32 master weights, fp32 gradients (exposed to the
  kernels as ``p.main_grad``), fp32 Adam moments.  Offsets are 64-element aligned so every
  kernel sees 16-byte aligned rows.  The order is reverse registration order, which is the order
  gradients complete in backward -- the data-parallel engine cuts its all-reduce buckets as
  contiguous ranges of this buffer, so no gradient is ever copied into a bucket.
* :class:`FusedAdamW` drives the ``adamw.hip`` kernels: global grad-norm (2 launches) + one
  multi-tensor AdamW launch, clip coefficient and 1/world folded in on the device, no host sync.
"""
from __future__ import annotations

import math
from typing import Dict, List, NamedTuple, Optional, Set, Tuple

import torch
import torch.nn as nn

ALIGN = 64
CHUNK = 32768


def param_groups(model: nn.Module) -> Tuple[Set[str], Set[str]]:
    decay, no_decay = set(), set()
    whitelist = (nn.Linear,)
    blacklist = (nn.LayerNorm, nn.Embedding)
    for mn, m in model.named_modules():
        for pn, p in m.named_parameters(recurse=False):
            fpn = f"{mn}.{pn}" if mn else pn
            if pn.endswith("bias"):
                no_decay.add(fpn)
            elif pn.endswith("weight") and isinstance(m, whitelist):
                decay.add(fpn)
            elif pn.endswith("weight") and isinstance(m, blacklist):
                no_decay.add(fpn)
            elif pn.endswith("in_proj_weight"):
                decay.add(fpn)
            elif pn.endswith("pos_embedding"):
                no_decay.add(fpn)
    params = dict(model.named_parameters())  # tied params appear once, under their first name
    # a tied weight (lm_head.weight is wte.weight) belongs to the group of its canonical name
    decay &= set(params)
    no_decay &= set(params)
    inter = decay & no_decay
    union = decay | no_decay
    assert not inter, f"parameters {inter} made it into both decay/no_decay sets!"
    missing = set(params) - union
    assert not missing, f"parameters {missing} were not separated into either decay/no_decay set!"
    return decay, no_decay


def create_optimizer(model: nn.Module, optimizer_config) -> torch.optim.AdamW:
    """Reference ``create_optimizer`` (two groups, wd / 0.0) as a torch AdamW."""
    decay, no_decay = param_groups(model)
    pd = dict(model.named_parameters())
    groups = [
        {"params": [pd[n] for n in sorted(decay)], "weight_decay": optimizer_config.weight_decay},
        {"params": [pd[n] for n in sorted(no_decay)], "weight_decay": 0.0},
    ]
    return torch.optim.AdamW(groups, lr=optimizer_config.learning_rate,
                             betas=tuple(optimizer_config.betas),
                             eps=getattr(optimizer_config, "eps", 1e-8))


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


class ChunkTable(NamedTuple):
    """Device chunk table of the multi-tensor kernels plus the bounds it was validated against:
    ``end`` = one past the last flat-buffer element any chunk touches, ``mend`` = the same for the
    (packed) moment buffers.  The bindings check the buffers they are handed against these, so a
    table built for another store (e.g. before a re-layout) fails loudly instead of indexing out
    of bounds."""
    start: torch.Tensor
    len: torch.Tensor
    wd: torch.Tensor
    mstart: torch.Tensor
    end: int
    mend: int


def make_chunk_table(pieces, device, bound: int, moment_bound: Optional[int] = None) -> ChunkTable:
    """Kernel chunk table from ``pieces`` = [(start, end, wd, moment_start)] of flat-buffer ranges:
    CHUNK-sized chunks (one workgroup each) that never straddle a piece, so weight decay is a
    per-chunk constant.  Every range is checked against the buffers here, on the host, because
    the kernels index the flat buffers through these tables unchecked."""
    starts, lens, wds, mstarts = [], [], [], []
    end = mend = 0
    for a, b, wd, ma in pieces:
        if not (0 <= a <= b <= bound) or a % 4 or (ma is not None and (ma % 4 or ma + (b - a) > moment_bound)):
            raise ValueError(f"chunk piece [{a}, {b}) (moments at {ma}) outside the flat buffers")
        end = max(end, b)
        mend = max(mend, (a if ma is None else ma) + (b - a))
        for c in range(a, b, CHUNK):
            starts.append(c)
            lens.append(min(CHUNK, b - c))
            wds.append(wd)
            mstarts.append(c - a + (a if ma is None else ma))
    t = dict(device=device)
    return ChunkTable(torch.tensor(starts, dtype=torch.int64, **t), torch.tensor(lens, dtype=torch.int32, **t),
                      torch.tensor(wds, dtype=torch.float32, **t), torch.tensor(mstarts, dtype=torch.int64, **t),
                      end, mend)


class FlatParamStore:
    """All parameters of ``model`` as views into flat buffers (see module docstring).

    ``bucket_numel`` cuts the layout into communication buckets: runs of whole parameters of at
    least that many elements, each padded to a multiple of ``bucket_align`` (the DP engine
    all-reduces a bucket as one contiguous slice; ZeRO-1 pads every bucket to ``world * 64`` so
    it splits into equal, aligned rank shards).  ``order`` (parameter names) fixes the layout
    order -- the data-parallel engine rebuilds the store in the order gradients were observed to
    complete -- and ``master_from`` initialises fp32 masters from another store by name."""

    def __init__(self, model: nn.Module, compute_dtype: Optional[torch.dtype] = None,
                 device: Optional[torch.device] = None, bucket_numel: Optional[int] = None,
                 bucket_align: int = ALIGN, order: Optional[List[str]] = None,
                 master_from: Optional["FlatParamStore"] = None):
        named = list(model.named_parameters())  # dedups tied weights
        if device is None:
            device = named[0][1].device
        device = torch.device(device)
        if compute_dtype is None:
            compute_dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
        if bucket_align % ALIGN:
            raise ValueError("bucket_align must be a multiple of 64 elements")
        self.device, self.compute_dtype = device, compute_dtype
        seq = list(reversed(named))  # reverse registration order ~ backward completion order
        if order is not None:
            rank = {n: k for k, n in enumerate(order)}
            seq.sort(key=lambda np_: rank.get(np_[0], len(rank)))  # stable: unknown names last
        self.names: List[str] = []
        self.params: List[nn.Parameter] = []
        self.offsets: List[int] = []
        self.numels: List[int] = []
        self.buckets: List[Tuple[int, int, List[int]]] = []
        off, bstart, cur = 0, 0, []
        for name, p in seq:
            if bucket_numel is not None and cur and p.numel() >= bucket_numel:
                # a parameter as large as a bucket gets a bucket of its own: the smaller
                # gradients before it launch without waiting for it (e.g. GPT-2's tied wte)
                off = _round_up(off, bucket_align)
                self.buckets.append((bstart, off, cur))
                bstart, cur = off, []
            self.names.append(name)
            self.params.append(p)
            self.offsets.append(off)
            self.numels.append(p.numel())
            off += _round_up(p.numel(), ALIGN)
            cur.append(len(self.params) - 1)
            if bucket_numel is not None and off - bstart >= bucket_numel:
                off = _round_up(off, bucket_align)
                self.buckets.append((bstart, off, cur))
                bstart, cur = off, []
        if cur or not self.buckets:
            off = _round_up(max(off, 1), bucket_align)
            self.buckets.append((bstart, off, cur))
        self.total = off
        f32 = dict(dtype=torch.float32, device=device)
        self.master = torch.zeros(self.total, **f32)
        self.grad = torch.zeros(self.total, **f32)
        src = {}
        if master_from is not None:
            src = {n: master_from.master[o:o + k] for n, o, k in
                   zip(master_from.names, master_from.offsets, master_from.numels)}
        for name, p, o, n in zip(self.names, self.params, self.offsets, self.numels):
            v = src.get(name)
            self.master[o:o + n].copy_(v if v is not None else
                                       p.detach().reshape(-1).to(device=device, dtype=torch.float32))
        if compute_dtype == torch.float32:
            self.flat = self.master  # CPU / fp32 path: params ARE the master weights
        else:
            self.flat = self.master.to(compute_dtype)
        for p, o, n in zip(self.params, self.offsets, self.numels):
            p.data = self.flat[o:o + n].view(p.shape)
            p.main_grad = self.grad[o:o + n].view(p.shape)
            p.grad = None
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        self.by_name: Dict[str, int] = {n: i for i, n in enumerate(self.names)}

    def views(self, buf: torch.Tensor) -> List[torch.Tensor]:
        return [buf[o:o + n].view(p.shape) for p, o, n in zip(self.params, self.offsets, self.numels)]

    def zero_grad(self):
        self.grad.zero_()

    def sync_params_from_master(self):
        if self.flat is not self.master:
            self.flat.copy_(self.master)

    def pieces(self, wd_of: Dict[str, float], lo: int = 0, hi: Optional[int] = None):
        """(start, end, wd) of every parameter's elements inside the flat range [lo, hi)."""
        hi = self.total if hi is None else hi
        out = []
        for name, o, n in zip(self.names, self.offsets, self.numels):
            a, b = max(o, lo), min(o + n, hi)
            if a < b:
                out.append((a, b, wd_of[name]))
        return out


class FusedAdamW:
    """AdamW over a :class:`FlatParamStore` (fp32 master weights, bf16 compute params)."""

    def __init__(self, store: FlatParamStore, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, decay_names: Optional[Set[str]] = None,
                 grad_clip: float = 0.0):
        self.store = store
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.grad_clip = grad_clip
        if decay_names is None:
            decay_names = {n for n, p in zip(store.names, store.params) if p.dim() >= 2}
        self.decay_names = set(decay_names)
        self.wd_of = {n: (weight_decay if n in self.decay_names else 0.0) for n in store.names}
        self.step_count = 0
        dev = store.device
        self.exp_avg = torch.zeros(store.total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(store.total, dtype=torch.float32, device=dev)
        self.norm_buf = torch.zeros(2, dtype=torch.float32, device=dev)
        pieces = [(a, b, wd, None) for a, b, wd in store.pieces(self.wd_of)]
        self.table = make_chunk_table(pieces, dev, store.total)
        self.n_chunks = int(self.table.len.numel())
        # where step() reads the (all-reduced) gradients: the fp32 main grads, or the bf16 buffer
        # the data-parallel engine reduced them in (DataParallelEngine(reduce_dtype=bf16))
        self.grad_buffer: torch.Tensor = store.grad
        # torch-optimizer look-alike for LR schedulers / logging
        self.param_groups = [{"lr": lr, "betas": self.betas, "weight_decay": weight_decay, "eps": eps}]

    @property
    def grad_norm(self) -> torch.Tensor:
        """Global grad norm of the last step (device tensor; read it lazily)."""
        return self.norm_buf[1]

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None, zero_grad: bool = False):
        """One AdamW step.  ``zero_grad``: also zero the fp32 main grads (on GPUs inside the update
        kernel, as each element is consumed: no separate fill pass)."""
        from .ops import streams

        streams.join()  # weight gradients still on the side stream (ops/streams.py)
        s = self.store
        lr = self.param_groups[0]["lr"] if lr is None else lr
        self.step_count += 1
        b1, b2 = self.betas
        if s.device.type == "cuda":
            from .ops._ext import ext

            C = ext()
            t = self.table
            C.grad_sumsq_chunks(t.start, t.len, self.grad_buffer, grad_scale, self.norm_buf, t.end)
            C.adamw_step(t.start, t.len, t.wd, None, s.master, s.flat, self.grad_buffer,
                         self.exp_avg, self.exp_avg_sq, self.norm_buf, lr, b1, b2, self.eps,
                         self.step_count, grad_scale, float(self.grad_clip), t.end, t.mend,
                         s.grad if zero_grad else None)
            return
        # CPU path (plain PyTorch, same math)
        g = self.grad_buffer.float() * grad_scale
        sumsq = (g * g).sum()
        self.norm_buf[0] = sumsq
        self.norm_buf[1] = sumsq.sqrt()
        if self.grad_clip > 0:
            coef = self.grad_clip / (self.norm_buf[1] + 1e-6)
            if coef < 1:
                g = g * coef
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        self.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        for name, o, n in zip(s.names, s.offsets, s.numels):
            wd = self.wd_of[name]
            sl = slice(o, o + n)
            if wd:
                s.master[sl].mul_(1 - lr * wd)
            denom = (self.exp_avg_sq[sl].sqrt() / math.sqrt(bc2)).add_(self.eps)
            s.master[sl].addcdiv_(self.exp_avg[sl], denom, value=-lr / bc1)
        s.sync_params_from_master()
        if zero_grad:
            s.zero_grad()

    # ------------------------------------------------------------------ state (by param name)
    def state_dict(self):
        s = self.store
        st = {}
        for name, o, n, p in zip(s.names, s.offsets, s.numels, s.params):
            st[name] = {"exp_avg": self.exp_avg[o:o + n].view(p.shape).cpu().clone(),
                        "exp_avg_sq": self.exp_avg_sq[o:o + n].view(p.shape).cpu().clone(),
                        "master": s.master[o:o + n].view(p.shape).cpu().clone()}
        return {"step": self.step_count, "state": st,
                "hparams": {"lr": self.param_groups[0]["lr"], "betas": list(self.betas), "eps": self.eps,
                            "weight_decay": self.weight_decay, "grad_clip": self.grad_clip}}

    def load_state_dict(self, sd):
        s = self.store
        self.step_count = int(sd["step"])
        for name, o, n in zip(s.names, s.offsets, s.numels):
            e = sd["state"].get(name)
            if e is None:
                continue
            self.exp_avg[o:o + n].copy_(e["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:o + n].copy_(e["exp_avg_sq"].reshape(-1))
            if "master" in e:
                s.master[o:o + n].copy_(e["master"].reshape(-1))
        s.sync_params_from_master()

    def zero_grad(self, set_to_none: bool = True):
        self.store.zero_grad()

    def rehome(self, new_store: FlatParamStore):
        """Move the moments to ``new_store``'s layout (same parameters, other order/padding)."""
        old = self.store

        def moved(buf):  # one new-layout buffer at a time: at most one extra moment buffer alive
            out = torch.zeros(new_store.total, dtype=torch.float32, device=new_store.device)
            for name, o, n in zip(old.names, old.offsets, old.numels):
                no = new_store.offsets[new_store.by_name[name]]
                out[no:no + n].copy_(buf[o:o + n])
            return out

        m = moved(self.exp_avg)
        self.exp_avg = None
        v = moved(self.exp_avg_sq)
        self.exp_avg_sq = None
        sd_step = self.step_count
        self.__init__(new_store, lr=self.param_groups[0]["lr"], betas=self.betas, eps=self.eps,
                      weight_decay=self.weight_decay, decay_names=self.decay_names,
                      grad_clip=self.grad_clip)
        self.exp_avg, self.exp_avg_sq, self.step_count = m, v, sd_step
