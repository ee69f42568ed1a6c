"""Process-group bootstrap and rank helpers (one process per GPU, torchrun env contract).

Replaces ``init_process_group("nccl")`` / ``LOCAL_RANK``/``RANK`` handling of the reference
(``/root/reference/mingpt/train.py:34,58``, ``trainer.py:53-54``) without its hard dependency on
torchrun env vars (D25): with no env it runs single-process.  On ROCm the ``nccl`` backend is
RCCL (collectives over xGMI between the GPUs of a node); ``gloo`` serves CPU runs and tests.
The device is bound with ``torch.cuda.set_device(local_rank)`` before the first collective (D24).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO = DistInfo()


def env_ranks():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_distributed(device: str = "auto", backend: str = "auto", timeout_s: int = 1800,
                     group_at_world1: bool = False) -> DistInfo:
    """Initialise (idempotent).  ``device``: auto|cuda|cpu.  ``backend``: auto|nccl|gloo.
    ``group_at_world1``: create a one-rank process group even without a torchrun env (drives the
    RCCL calls on one GPU: plumbing checks of the collective path, ``comm_at_world1`` engines)."""
    global _INFO
    rank, world, local = env_ranks()
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    if device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if backend == "auto":
        backend = "nccl" if dev.type == "cuda" else "gloo"
    if (world > 1 or group_at_world1) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            import socket

            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        restart = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if restart > 0 and "MASTER_PORT" in os.environ:
            # A restarted worker group shares torchrun's store with the dead one; without a
            # per-attempt prefix a rank can read a dead peer's gloo address / RCCL unique id
            # and fail to connect (or hang).  Namespace the bootstrap keys by attempt.
            agent_store = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                                 is_master=(rank == 0 and not agent_store), timeout=kw["timeout"])
            kw.update(store=dist.PrefixStore(f"mingpt/attempt{restart}", base), rank=rank, world_size=world)
        dist.init_process_group(**kw)
    _INFO = DistInfo(rank=rank, world_size=world, local_rank=local, device=dev,
                     backend=backend if (world > 1 or dist.is_initialized()) else "none")
    return _INFO


def info() -> DistInfo:
    return _INFO


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world_size() -> int:
    """Ranks in the default process group (1 when none was created)."""
    return dist.get_world_size() if is_initialized() else 1


def barrier():
    if is_initialized():
        dist.barrier()


def all_reduce_mean(t: torch.Tensor) -> torch.Tensor:
    """Average a (small) tensor over ranks, e.g. the logged loss (fixes D23: rank-local loss)."""
    if is_initialized() and dist.get_world_size() > 1:
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= dist.get_world_size()
    return t


def all_reduce_max(x: float, device) -> float:
    if is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return x


def destroy():
    if is_initialized():
        dist.destroy_process_group()
