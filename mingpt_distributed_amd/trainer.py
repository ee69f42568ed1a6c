"""Training runtime.

Two front-ends over one step engine:

* :class:`GPTTrainer` / :class:`GPTTrainerConfig` / :class:`ModelSnapshot` -- the reference's
  epoch-based distributed trainer (``/root/reference/mingpt/trainer.py:21-183``): DP across GPUs,
  rank-sharded sampler, grad clipping, periodic loss log, test epoch, snapshot save/resume to a
  local path or ``s3://`` (fsspec reads, boto3 upload).  The reference's defects are fixed:
  D15-D17 (wrong method/attribute names), D18 (resume re-trained the saved epoch), D19 (snapshot
  written by every node's local rank 0: now global rank 0, atomic temp+rename), D20
  (``set_epoch``), D21 (``eval()`` for the test epoch), D22 (grad norm logged), D23 (loss
  all-reduced before logging, read from the device only every ``log_every`` batches),
  D25 (runs without torchrun env).
* :class:`Trainer` -- the upstream-minGPT iteration API the reference README advertises
  (``get_default_config``, ``add_callback('on_batch_end', fn)``, ``run()``, ``iter_num`` /
  ``iter_dt`` / ``loss``).

:class:`StepEngine` is the MI355X part: bf16 compute params + fp32 master/grads in flat buffers,
fused HIP kernels for forward/backward, :class:`DataParallelEngine` overlapping the bucketed
RCCL all-reduce with backward, :class:`FusedAdamW` (clip + 1/world folded in on the device).
"""
from __future__ import annotations

import contextlib
import io
import os
import shutil
import time
from collections import defaultdict
from dataclasses import asdict, dataclass
from typing import Any, Dict, List, Optional

import torch
from torch.utils.data import DataLoader, Dataset

from .ops import streams
from .optim import FlatParamStore, FusedAdamW, param_groups
from .parallel import dist as D
from .parallel.ddp import DataParallelEngine
from .parallel.sampler import DistributedSampler, InfiniteRandomSampler
from .utils.config import CfgNode


# ====================================================================================== engine
_ROCTX = os.environ.get("MINGPT_ROCTX", "0") not in ("", "0")


def _fold_grad(p):
    if p.grad is not None:
        p.main_grad.add_(p.grad.to(p.main_grad.dtype))
        p.grad = None


class StepEngine:
    def __init__(self, model: torch.nn.Module, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, grad_clip: float = 1.0, decay_names=None,
                 device: Optional[torch.device] = None, bucket_mb: float = 32.0, reduce_dtype=None,
                 zero1: bool = False, comm_at_world1: bool = False, comm: Optional[str] = None):
        """``reduce_dtype``: None (fp32 gradients on the wire) or ``torch.bfloat16``.
        ``zero1``: shard the AdamW state over the data-parallel ranks (also valid at world 1).
        ``comm_at_world1``: drive the collectives even in a one-rank process group (tests).
        ``comm``: ``c10d`` or ``rccl`` (the engines' own RCCL communicator, parallel/comm.py);
        default ``MINGPT_COMM`` or c10d."""
        if device is None:
            info = D.info()
            if info.device.type == "cuda":
                device = info.device
            elif torch.cuda.is_available():
                device = torch.device("cuda", torch.cuda.current_device())
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        if self.device.type == "cuda" and hasattr(getattr(model, "config", None), "check_gpu_support"):
            model.config.check_gpu_support()  # fail at construction, not inside the first step
        self.model = model.to(self.device)
        if decay_names is None:
            decay_names, _ = param_groups(model)
        multi = D.is_initialized() and (torch.distributed.get_world_size() > 1 or comm_at_world1)
        world = torch.distributed.get_world_size() if multi else 1
        self.comm_at_world1 = comm_at_world1
        self.comm = comm
        if reduce_dtype == "auto":
            reduce_dtype = None
        self.zero1 = bool(zero1)
        self._okw = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decay_names=decay_names,
                         grad_clip=grad_clip or 0.0)
        self.bucket_mb, self.reduce_dtype = bucket_mb, reduce_dtype
        bucket_numel = DataParallelEngine.bucket_numel(bucket_mb) if (multi or zero1) else None
        if self.zero1:  # optimizer state sharded over the ranks (parallel/zero.py)
            from .parallel.zero import ZeroAdamW, ZeroGradEngine

            self.store = FlatParamStore(model, device=self.device, bucket_numel=bucket_numel,
                                        bucket_align=64 * world)
            self.dp = ZeroGradEngine(self.store, reduce_dtype=reduce_dtype, model=model,
                                     comm_at_world1=comm_at_world1, comm=comm)
            self.opt = ZeroAdamW(self.store, self.dp, **self._okw)
        else:
            self.store = FlatParamStore(model, device=self.device, bucket_numel=bucket_numel)
            self.opt = FusedAdamW(self.store, **self._okw)
            self.dp = DataParallelEngine(self.store, bucket_mb=bucket_mb, reduce_dtype=reduce_dtype,
                                         comm_at_world1=comm_at_world1, comm=comm) if multi else None
            if self.dp is not None:
                self.opt.grad_buffer = self.dp.grad_buffer
        self.world = self.dp.world if self.dp else 1
        self._hooks = []
        self.annotate = False  # record_function ranges (fwd/bwd/allreduce/optim) while profiling
        self.measure_comm = False  # hipEvents around dp.finish() (comm_exposed_ms)
        self._comm_events = []
        self._fold_hooks()
    def _fold_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self.dp is None or not self.dp.active:
            # single process: ops that return ordinary autograd grads (the CPU reference path)
            # are folded into the fp32 main-grad buffer the optimizer reads
            for p in self.store.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(_fold_grad))

    def _relayout(self, order):
        """Rebuild the flat buffers (and so the all-reduce buckets) in ``order`` -- the gradient
        completion order the data-parallel engine observed in the first backward -- keeping
        fp32 masters and Adam moments (DDP's bucket rebuild after iteration 1)."""
        old_store, old_dp = self.store, self.dp
        old_dp.close()
        old_dp.comm = None  # its bf16 reduce buffer; the new engine allocates its own
        # transient memory: the old gradient buffer holds nothing needed after the optimizer step
        # (the new store starts from zero grads), so it goes first; the moments are moved one
        # buffer at a time (FusedAdamW.rehome)
        old_store.grad = None
        for p in old_store.params:
            p.main_grad = None
        new = FlatParamStore(self.model, device=self.device,
                             bucket_numel=DataParallelEngine.bucket_numel(self.bucket_mb),
                             order=order, master_from=old_store)
        old_store.master = old_store.flat = None  # copied into `new`; only its layout is read below
        self.opt.rehome(new)
        self.store = new
        native = self.dp.native if self.dp is not None else None  # the communicator outlives the layout
        self.dp = DataParallelEngine(new, bucket_mb=self.bucket_mb, reduce_dtype=self.reduce_dtype,
                                     broadcast=False, comm_at_world1=self.comm_at_world1, comm=self.comm,
                                     native=native, proxy=self.dp.proxy)
        self.dp.observed = None
        self.dp._recording = None
        self.opt.grad_buffer = self.dp.grad_buffer
        self._graph = None

    @classmethod
    def from_torch_optimizer(cls, model, optimizer: torch.optim.Optimizer, grad_clip: float, **kw):
        """Adopt the hyper-parameters of a torch AdamW built by ``create_optimizer``."""
        g0 = optimizer.param_groups[0]
        names = {id(p): n for n, p in model.named_parameters()}
        decay = set()
        wd = 0.0
        for g in optimizer.param_groups:
            if g.get("weight_decay", 0.0) > 0:
                wd = g["weight_decay"]
                decay |= {names[id(p)] for p in g["params"] if id(p) in names}
        return cls(model, lr=g0["lr"], betas=g0["betas"], eps=g0.get("eps", 1e-8), weight_decay=wd,
                   grad_clip=grad_clip, decay_names=decay, **kw)

    @property
    def lr(self):
        return self.opt.param_groups[0]["lr"]

    @lr.setter
    def lr(self, v):
        self.opt.param_groups[0]["lr"] = v

    def to_device(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self.device, non_blocking=True)

    def _range(self, name: str):
        if _ROCTX and self.device.type == "cuda":
            # roctx ranges (torch.cuda.nvtx is roctx on ROCm): step phases show up as named
            # ranges in `rocprofv3 --marker-trace` next to the kernel trace
            return torch.cuda.nvtx.range(name)
        return torch.profiler.record_function(name) if self.annotate else contextlib.nullcontext()

    def forward_backward(self, x, y, scale: float = 1.0, sync: bool = True):
        ctx = self.dp.no_sync() if (self.dp is not None and not sync) else contextlib.nullcontext()
        width = getattr(getattr(self.model, "config", None), "n_embd", None)
        with ctx, streams.compute_stream(self.device, x.numel(), width):
            with self._range("mingpt::forward"):
                _, loss = self.model(x, y)
            with self._range("mingpt::backward"):
                (loss * scale if scale != 1.0 else loss).backward()
                streams.join()  # the block weight gradients ran on the side stream
            if self.dp is not None:
                ev = None
                if self.measure_comm and sync and self.device.type == "cuda":
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record()  # after the last backward kernel on the compute stream
                with self._range("mingpt::allreduce_wait"):
                    self.dp.finish()
                if ev is not None:
                    ev[1].record()  # the compute stream has waited for every outstanding collective
                    self._comm_events.append(ev)
        return loss.detach()

    def comm_exposed_ms(self, reset: bool = True) -> Optional[float]:
        """Mean device time, over the synchronised steps since the last call, from the end of
        backward's last kernel to the end of ``dp.finish()`` (the gradient communication NOT
        hidden under backward).  Needs ``measure_comm = True`` beforehand; synchronises the
        device; None when nothing was recorded (no data-parallel engine, CPU)."""
        evs = self._comm_events
        if reset:
            self._comm_events = []
        if not evs:
            return None
        torch.cuda.synchronize(self.device)
        return sum(a.elapsed_time(b) for a, b in evs) / len(evs)

    def optimizer_step(self):
        with self._range("mingpt::optimizer"):
            if not self.zero1:  # replicated AdamW zeroes the grads inside its update kernel
                self.opt.step(grad_scale=1.0 / self.world, zero_grad=True)
            else:
                self.opt.step(grad_scale=1.0 / self.world)
                self.store.zero_grad()
        if self.dp is not None:
            order = self.dp.relayout_order()
            if order is not None:
                self._relayout(order)

    def train_step(self, batches) -> torch.Tensor:
        """One optimizer step over a list of (x, y) micro-batches; returns the mean loss (device)."""
        n = len(batches)
        total = None
        for i, (x, y) in enumerate(batches):
            l = self.forward_backward(self.to_device(x), self.to_device(y), scale=1.0 / n, sync=(i == n - 1))
            total = l if total is None else total + l
        self.optimizer_step()
        return total / n

    def train_step_local(self, batches) -> torch.Tensor:
        """``train_step`` with every gradient collective skipped: each rank updates its replica
        from its OWN gradients (diagnostics only -- the replicas diverge).  bench.py times it at
        N > 1 to split the 1 -> N step-time loss into exposed communication and compute slowed
        by the node's other ranks.  Replicated DP only (ZeRO-1's update needs the reduce-scatter)."""
        if self.zero1:
            raise RuntimeError("train_step_local: ZeRO-1's sharded update needs reduced gradients")
        n = len(batches)
        total = None
        for x, y in batches:
            l = self.forward_backward(self.to_device(x), self.to_device(y), scale=1.0 / n, sync=False)
            total = l if total is None else total + l
        gb, self.opt.grad_buffer = self.opt.grad_buffer, self.store.grad  # the local fp32 grads
        try:
            self.optimizer_step()
        finally:
            self.opt.grad_buffer = gb
        return total / n

    # ------------------------------------------------------------------ hipGraph step
    def graph_step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """``train_step([(x, y)])`` as ONE hipGraph replay (single process, GPU).

        The whole step -- embedding, every block's fused kernels, head + loss, backward, grad-norm,
        AdamW, grad zeroing -- is captured once per input shape and replayed: one launch per step
        instead of ~20 per layer from Python, which is what bounds small models (chargpt's
        gpt-mini at T=128 is launch-bound) and removes host jitter for large ones.  What changes
        per step lives in device memory: the inputs (copied into static buffers), a dropout seed
        counter bumped inside the graph (common.h eff_seed: every replay draws new masks), and
        AdamW's {lr, step} written before each replay.  Returns the step's loss (a static buffer,
        overwritten by the next replay)."""
        if self.device.type != "cuda" or self.dp is not None:
            return self.train_step([(x, y)])
        from .ops._ext import ext

        C = ext()
        key = (tuple(x.shape), tuple(y.shape))
        g = getattr(self, "_graph", None)
        if g is None or g["key"] != key:
            g = self._capture(C, key, x, y)
        g["x"].copy_(x, non_blocking=True)
        g["y"].copy_(y, non_blocking=True)
        self.opt.step_count += 1
        g["hp"][0].fill_(float(self.opt.param_groups[0]["lr"]))
        g["hp"][1].fill_(float(self.opt.step_count))
        g["graph"].replay()
        return g["loss"]

    def _capture(self, C, key, x, y):
        self._graph = None
        dev = self.device
        st = {"key": key, "x": torch.empty_like(x, device=dev), "y": torch.empty_like(y, device=dev),
              "hp": torch.zeros(2, dtype=torch.float32, device=dev),
              "seed": torch.zeros(1, dtype=torch.int64, device=dev)}
        st["x"].copy_(x)
        st["y"].copy_(y)
        # warm up on a side stream (allocator / autograd state), as torch.cuda.graph requires;
        # these are real optimizer steps, so they count
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                self.train_step([(st["x"], st["y"])])
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        C.set_graph_state(st["seed"], st["hp"])
        n0 = self.opt.step_count
        try:
            with torch.cuda.graph(graph):
                st["seed"].add_(1)
                st["loss"] = self.train_step([(st["x"], st["y"])])
        finally:
            C.set_graph_state(None, None)
            self.opt.step_count = n0  # the captured step ran no update; replays advance it
        st["graph"] = graph
        self._graph = st
        return st

    @property
    def grad_norm(self) -> torch.Tensor:
        return self.opt.grad_norm

    def model_state_dict(self) -> Dict[str, torch.Tensor]:
        """fp32 CPU state dict (master weights for parameters)."""
        s = self.store
        masters = {id(p): s.master[o:o + n].view(p.shape) for p, o, n in zip(s.params, s.offsets, s.numels)}
        out = {}
        for k, v in self.model.state_dict(keep_vars=True).items():
            src = masters.get(id(v), v)
            out[k] = src.detach().float().cpu().clone() if src.is_floating_point() else src.detach().cpu().clone()
        return out

    def load_model_state_dict(self, sd: Dict[str, torch.Tensor]):
        s = self.store
        named = dict(self.model.named_parameters())
        for name, p in named.items():
            if name in sd:
                i = s.index[id(p)]
                o, n = s.offsets[i], s.numels[i]
                s.master[o:o + n].copy_(sd[name].reshape(-1).to(s.master.device, torch.float32))
        for name, b in self.model.named_buffers():
            if name in sd:
                b.copy_(sd[name])
        s.sync_params_from_master()


# ====================================================================================== snapshots
@dataclass
class GPTTrainerConfig:
    max_epochs: Optional[int] = None
    batch_size: Optional[int] = None
    learning_rate: Optional[float] = None   # unused, as in the reference (LR lives in OptimizerConfig)
    grad_norm_clip: Optional[float] = None
    dl_num_workers: Optional[int] = 0
    snapshot_path: Optional[str] = None
    save_every: Optional[int] = 1
    # extensions
    log_every: int = 100
    grad_accum_steps: int = 1
    max_steps_per_epoch: Optional[int] = None
    seed: int = 0
    save_every_steps: Optional[int] = None      # step-granular snapshots (mid-epoch resume)
    zero1: bool = False                         # shard AdamW state over the ranks (parallel/zero.py)
    fault_inject_step: Optional[int] = None     # test hook: fail after this global step
    fault_inject_rank: Optional[int] = None     # ... on this rank only (None = every rank)
    fault_inject_mode: str = "raise"            # "raise" (InjectedFault) or "exit" (os._exit(13))
    metrics_path: Optional[str] = None          # rank-0 JSONL: loss, tokens/s, MFU, grad_norm, lr
    profile_dir: Optional[str] = None           # torch.profiler (roctracer) trace of a step window
    profile_steps: str = "3:6"                  # [start, end) global steps traced
    peak_tflops: float = 2500.0                 # per-GPU dense bf16 peak used for MFU


class InjectedFault(RuntimeError):
    """Raised by ``fault_inject_step``: a deterministic worker failure to test resume."""


@dataclass
class ModelSnapshot:
    """Reference schema (``/root/reference/mingpt/trainer.py:33-37``) plus step-granular state.

    ``final_epoch`` is the epoch the snapshot was taken in; ``epoch_step`` > 0 marks a mid-epoch
    snapshot (that many optimizer steps of ``final_epoch`` done), 0 a completed epoch.
    ``rng_state`` is torch's CPU generator (dropout seeds and data order derive from it)."""
    model_state: "Dict[str, torch.Tensor]"
    optimizer_state: Dict[str, Any]
    final_epoch: int
    step: int = 0
    epoch_step: int = 0
    rng_state: Optional[torch.Tensor] = None


def _is_local(fs) -> bool:
    proto = fs.protocol if isinstance(fs.protocol, str) else fs.protocol[0]
    return proto in ("file", "local")


def _atomic_save(obj, path: str):
    """Crash-safe snapshot write (replaces the reference's plain ``torch.save``,
    ``/root/reference/mingpt/trainer.py:149-167``).

    1. the bytes go to ``path.tmp`` (fsynced on a local / Lustre path);
    2. the current snapshot, if any, is kept as ``path.prev`` (a hard link where the filesystem
       has them, else a copy) -- ``path`` itself is never removed;
    3. ``path.tmp`` replaces ``path`` by one atomic rename (``os.replace``); object stores, whose
       ``mv`` has no rm window to begin with, go through fsspec.

    A crash at any point leaves ``path`` (old or new, never torn or missing) or, at worst, the
    previous snapshot in ``path.prev``, which ``GPTTrainer._load_snapshot`` falls back to."""
    import fsspec

    fs, p = fsspec.core.url_to_fs(path)
    tmp, prev = p + ".tmp", p + ".prev"
    buf = io.BytesIO()
    torch.save(obj, buf)
    if _is_local(fs):
        d = os.path.dirname(os.path.abspath(p))
        os.makedirs(d, exist_ok=True)
        with open(tmp, "wb") as f:
            f.write(buf.getvalue())
            f.flush()
            os.fsync(f.fileno())
        if os.path.exists(p):
            if os.path.lexists(prev):
                os.remove(prev)
            try:
                os.link(p, prev)
            except OSError:  # no hard links here (some network filesystems): copy
                shutil.copyfile(p, prev)
        os.replace(tmp, p)
        try:  # persist the rename itself
            fd = os.open(d, os.O_RDONLY)
            try:
                os.fsync(fd)
            finally:
                os.close(fd)
        except OSError:
            pass
        return
    with fs.open(tmp, "wb") as f:
        f.write(buf.getvalue())
    if fs.exists(p):
        fs.copy(p, prev)
    fs.mv(tmp, p)


class GPTTrainer:
    """Reference-API distributed trainer (see module docstring)."""

    s3_client_factory = None  # test seam: callable returning an object with upload_fileobj()

    def __init__(self, config: GPTTrainerConfig, model: torch.nn.Module, optimizer: Any,
                 train_dataset: Dataset, test_dataset: Optional[Dataset] = None):
        info = D.info() if D.is_initialized() else D.init_distributed()
        self.local_rank, self.global_rank, self.world = info.local_rank, info.rank, info.world_size
        self.config = config
        self.train_dataset, self.test_dataset = train_dataset, test_dataset
        self.train_loader = self._prepare_dataloader(train_dataset)
        self.test_loader = self._prepare_dataloader(test_dataset, shuffle=False) if test_dataset else None
        if self.config.snapshot_path is None:
            self.config.snapshot_path = "gpt_snapshot.pt"
        clip = config.grad_norm_clip or 0.0
        if isinstance(optimizer, torch.optim.Optimizer):
            self.engine = StepEngine.from_torch_optimizer(model, optimizer, clip, zero1=config.zero1)
        else:
            self.engine = StepEngine(model, grad_clip=clip, zero1=config.zero1)
        self.model = self.engine.model
        self.optimizer = self.engine.opt
        self.save_every = config.save_every or 1
        self.last_epoch = -1
        self.step = 0
        self.resume_epoch_step = 0
        self.history: List[Dict[str, float]] = []
        self._metrics_f = None
        self._prof = None
        self._pending_rng = None
        self._flops_per_token = model.flops_per_token() if hasattr(model, "flops_per_token") else None
        self._load_snapshot()

    # ------------------------------------------------------------------ data
    def _prepare_dataloader(self, dataset: Dataset, shuffle: bool = True):
        sampler = DistributedSampler(dataset, num_replicas=self.world, rank=self.global_rank,
                                     shuffle=shuffle, seed=self.config.seed)
        return DataLoader(dataset, batch_size=self.config.batch_size, sampler=sampler,
                          pin_memory=torch.cuda.is_available(), shuffle=False,
                          num_workers=self.config.dl_num_workers or 0, drop_last=True)

    # ------------------------------------------------------------------ snapshots
    def _snapshot_dict(self, epoch: int, epoch_step: int = 0) -> Dict[str, Any]:
        snap = ModelSnapshot(model_state=self.engine.model_state_dict(),
                             optimizer_state=self.engine.opt.state_dict(), final_epoch=epoch,
                             step=self.step, epoch_step=epoch_step, rng_state=torch.get_rng_state())
        return asdict(snap)

    def _upload_snapshot(self, snapshot, dst: str):
        from urllib.parse import urlparse

        buffer = io.BytesIO()
        torch.save(snapshot, buffer)
        buffer.seek(0)
        u = urlparse(dst, allow_fragments=False)
        if self.s3_client_factory is not None:
            client = self.s3_client_factory()
        else:
            import boto3  # lazy: only needed for s3:// snapshots

            client = boto3.client("s3")
        client.upload_fileobj(buffer, u.netloc, u.path.lstrip("/"))

    def _consolidate(self) -> None:
        # ZeRO-1: masters and moments are sharded; gather them on every rank before rank 0 saves
        if hasattr(self.engine.opt, "consolidate"):
            self.engine.opt.consolidate()

    def _save_snapshot(self, epoch: int, epoch_step: int = 0) -> None:
        # every rank must take part in nothing here: called on global rank 0 only (D19)
        snapshot = self._snapshot_dict(epoch, epoch_step)
        path = self.config.snapshot_path
        if path.startswith("s3://"):
            self._upload_snapshot(snapshot, path)
        else:
            _atomic_save(snapshot, path)
        where = f"epoch {epoch}" + (f" step {epoch_step}" if epoch_step else "")
        print(f"Model snapshot taken and saved at {where}")

    def _load_snapshot(self):
        import fsspec

        # the snapshot, else the one _atomic_save kept before it (a crash inside a save, or a
        # snapshot that no longer loads); nothing found at either: train from scratch
        data, errors = None, []
        for cand in (self.config.snapshot_path, self.config.snapshot_path + ".prev"):
            try:
                with fsspec.open(cand, "rb") as f:
                    data = torch.load(f, map_location="cpu", weights_only=True)
            except FileNotFoundError:
                continue
            except Exception as e:  # torn / unreadable file: try the previous one
                errors.append(f"{cand}: {type(e).__name__}: {e}")
                continue
            if cand != self.config.snapshot_path and self.global_rank == 0:
                print(f"Snapshot {self.config.snapshot_path} missing or unreadable; resuming from {cand}")
            break
        if data is None:
            if errors:  # snapshots exist but none loads: never silently start over
                raise RuntimeError("no loadable snapshot: " + "; ".join(errors))
            if self.global_rank == 0:
                print("Model snapshot not found. Training from scratch.")
            return
        snap = ModelSnapshot(**data)
        self.engine.load_model_state_dict(snap.model_state)
        self.engine.opt.load_state_dict(snap.optimizer_state)
        self.step = snap.step
        # applied once the resumed epoch's DataLoader iterator exists (creating it draws a seed)
        self._pending_rng = snap.rng_state
        if snap.epoch_step > 0:  # mid-epoch snapshot: finish that epoch first
            self.last_epoch = snap.final_epoch - 1
            self.resume_epoch_step = snap.epoch_step
        else:
            self.last_epoch = snap.final_epoch
        if self.global_rank == 0:
            print(f"Resuming training from epoch {self.last_epoch + 1}"
                  + (f" step {self.resume_epoch_step}" if self.resume_epoch_step else ""))

    # ------------------------------------------------------------------ observability
    def _log_metrics(self, rec: Dict[str, Any]) -> None:
        if self.global_rank != 0 or not self.config.metrics_path:
            return
        import json

        if self._metrics_f is None:
            d = os.path.dirname(self.config.metrics_path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._metrics_f = open(self.config.metrics_path, "a")
        self._metrics_f.write(json.dumps(rec) + "\n")
        self._metrics_f.flush()

    def _profile_tick(self) -> None:
        """Start/stop a torch.profiler window over global steps [start, end) (rank 0)."""
        if not self.config.profile_dir or self.global_rank != 0:
            return
        a, b = (int(v) for v in self.config.profile_steps.split(":"))
        if self.step == a and self._prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if self.engine.device.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()
            self.engine.annotate = True
        elif self.step == b and self._prof is not None:
            self._prof.__exit__(None, None, None)
            self.engine.annotate = False
            os.makedirs(self.config.profile_dir, exist_ok=True)
            self._prof.export_chrome_trace(os.path.join(self.config.profile_dir, "trace.json"))
            sort = "cuda_time_total" if self.engine.device.type == "cuda" else "cpu_time_total"
            with open(os.path.join(self.config.profile_dir, "summary.txt"), "w") as f:
                f.write(self._prof.key_averages().table(sort_by=sort, row_limit=50))
            self._prof = None

    def _maybe_inject_fault(self) -> None:
        c = self.config
        if c.fault_inject_step is None or self.step != c.fault_inject_step:
            return
        if c.fault_inject_rank is not None and c.fault_inject_rank != self.global_rank:
            return
        if int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0:
            return  # the restarted worker group runs clean (elastic-recovery test)
        print(f"[GPU{self.global_rank}] injected fault after step {self.step}", flush=True)
        if c.fault_inject_mode == "exit":
            os._exit(13)  # a hard worker death: torchrun sees a failed rank
        raise InjectedFault(f"injected fault after step {self.step}")

    # ------------------------------------------------------------------ loops
    def _run_batch(self, inputs, labels, train: bool = True) -> torch.Tensor:
        if train:
            return self.engine.train_step([(inputs, labels)])
        with torch.no_grad():
            _, loss = self.model(self.engine.to_device(inputs), self.engine.to_device(labels))
        return loss.detach()

    def _run_epoch(self, epoch: int, dataloader: DataLoader, train: bool = True) -> float:
        skip = self.resume_epoch_step if train else 0
        if isinstance(dataloader.sampler, DistributedSampler):
            dataloader.sampler.set_epoch(epoch, start=skip * (self.config.batch_size or 1))
        self.model.train(train)
        total, count = None, 0
        t0 = tlog = time.perf_counter()
        nlog = 0
        c = self.config
        it = iter(dataloader)
        if train and self._pending_rng is not None:
            torch.set_rng_state(self._pending_rng)
            self._pending_rng = None
        for i, (x, y) in enumerate(it):
            idx = i + skip
            if train and c.max_steps_per_epoch and idx >= c.max_steps_per_epoch:
                break
            if train:
                self._profile_tick()
            loss = self._run_batch(x, y, train)
            total = loss if total is None else total + loss
            count += 1
            nlog += 1
            if train:
                self.step += 1
                if c.save_every_steps and self.step % c.save_every_steps == 0:
                    self._consolidate()
                    if self.global_rank == 0:
                        self._save_snapshot(epoch, epoch_step=idx + 1)
                self._maybe_inject_fault()
            if idx % c.log_every == 0:
                lg = D.all_reduce_mean(loss.float()).item()   # syncs the device: timing is honest
                now = time.perf_counter()
                if self.global_rank == 0:
                    dt = now - tlog
                    tok_s = x.numel() * self.world * nlog / max(dt, 1e-9)
                    gn = self.engine.grad_norm.item() if train else float("nan")
                    print(f"[GPU{self.global_rank}] Epoch {epoch} | Iter {idx} | "
                          f"{'Training' if train else 'Test'} loss {lg:.5f} | grad_norm {gn:.3f} | "
                          f"{tok_s:,.0f} tok/s", flush=True)
                    rec = {"epoch": epoch, "iter": idx, "step": self.step, "split": "train" if train else "test",
                           "loss": lg, "tokens_per_s": tok_s, "step_ms": dt / nlog * 1e3}
                    if train:
                        rec.update(grad_norm=gn, lr=self.engine.lr)
                        if self._flops_per_token and self.engine.device.type == "cuda":
                            rec["mfu"] = tok_s * self._flops_per_token / (self.world * c.peak_tflops * 1e12)
                    self._log_metrics(rec)
                tlog, nlog = now, 0
        if train:
            self.resume_epoch_step = 0
        if count == 0:
            return float("nan")
        mean = D.all_reduce_mean((total / count).float()).item()
        self.model.train(True)
        return mean

    def train(self) -> None:
        start = self.last_epoch + 1
        try:
            for epoch in range(start, self.config.max_epochs):
                tr = self._run_epoch(epoch, self.train_loader, True)
                rec = {"epoch": epoch, "train_loss": tr}
                if epoch % self.save_every == 0:
                    self._consolidate()
                    if self.global_rank == 0:
                        self._save_snapshot(epoch)
                if self.test_loader is not None:
                    rec["test_loss"] = self._run_epoch(epoch, self.test_loader, False)
                self.history.append(rec)
                self._log_metrics(dict(rec, split="epoch"))
                D.barrier()
        finally:
            if self._prof is not None:
                self._prof.__exit__(None, None, None)
                self._prof = None
            if self._metrics_f is not None:
                self._metrics_f.close()
                self._metrics_f = None


# ====================================================================================== upstream
class Trainer:
    """Upstream-minGPT iteration trainer API, on the MI355X step engine."""

    @staticmethod
    def get_default_config() -> CfgNode:
        C = CfgNode()
        C.device = "auto"
        C.num_workers = 4
        C.max_iters = None
        C.batch_size = 64
        C.learning_rate = 3e-4
        C.betas = (0.9, 0.95)
        C.weight_decay = 0.1
        C.grad_norm_clip = 1.0
        C.grad_accum_steps = 1
        C.cuda_graph = False  # replay each step as one hipGraph (StepEngine.graph_step; 1 GPU)
        return C

    def __init__(self, config, model, train_dataset):
        self.config = config
        self.model = model
        self.train_dataset = train_dataset
        self.callbacks = defaultdict(list)
        dev = config.device
        if dev == "auto":
            dev = "cuda" if torch.cuda.is_available() else "cpu"
        if not D.is_initialized():
            D.init_distributed(device=dev)
        self.device = dev
        print("running on device", self.device)
        decay, _ = param_groups(model)
        self.engine = StepEngine(model, lr=config.learning_rate, betas=config.betas,
                                 weight_decay=config.weight_decay, grad_clip=config.grad_norm_clip,
                                 decay_names=decay,
                                 device=D.info().device if dev == "cuda" else torch.device("cpu"))
        self.optimizer = self.engine.opt
        self.iter_num = 0
        self.iter_time = 0.0
        self.iter_dt = 0.0
        self.loss = None

    def add_callback(self, onevent: str, callback):
        self.callbacks[onevent].append(callback)

    def set_callback(self, onevent: str, callback):
        self.callbacks[onevent] = [callback]

    def trigger_callbacks(self, onevent: str):
        for callback in self.callbacks.get(onevent, []):
            callback(self)

    def run(self):
        model, config = self.model, self.config
        info = D.info()
        loader = DataLoader(self.train_dataset,
                            sampler=InfiniteRandomSampler(self.train_dataset, rank=info.rank),
                            shuffle=False, pin_memory=self.device == "cuda", batch_size=config.batch_size,
                            num_workers=config.num_workers)
        model.train()
        self.iter_num = 0
        self.iter_time = time.time()
        data_iter = iter(loader)
        accum = max(1, getattr(config, "grad_accum_steps", 1))
        graph = bool(getattr(config, "cuda_graph", False)) and accum == 1
        while True:
            batches = [next(data_iter) for _ in range(accum)]
            if graph:
                self.loss = self.engine.graph_step(*batches[0])
            else:
                self.loss = self.engine.train_step(batches)
            self.trigger_callbacks("on_batch_end")
            self.iter_num += 1
            tnow = time.time()
            self.iter_dt = tnow - self.iter_time
            self.iter_time = tnow
            if config.max_iters is not None and self.iter_num >= config.max_iters:
                break
