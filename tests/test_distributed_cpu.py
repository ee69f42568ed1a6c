"""Multi-process data parallelism on CPU (gloo, world_size 2): the same engine code that drives
RCCL on the GPUs.  Checks: the 2-rank step equals the 1-process step on the concatenated batch,
parameters stay bit-identical across ranks, gradient accumulation (no_sync), GPTTrainer with
rank-0-only snapshots."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from mingpt_distributed_amd.parallel import dist as D

    return D.init_distributed(device="cpu", backend="gloo")


def _model():
    from mingpt_distributed_amd.models import GPT, GPTConfig

    torch.manual_seed(0)
    return GPT(GPTConfig(n_layer=2, n_head=2, n_embed=32, vocab_size=50, block_size=16, embed_drop=0.0,
                         resid_drop=0.0, attn_drop=0.0), verbose=False)


def _batch():
    g = torch.Generator().manual_seed(1)
    return torch.randint(0, 50, (4, 16), generator=g), torch.randint(0, 50, (4, 16), generator=g)


def _worker_dp(rank, world, port, out_dir, accum, bf16=False):
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, bucket_mb=0.01,  # tiny buckets: many collectives
                     reduce_dtype=torch.bfloat16 if bf16 else None)
    assert eng.dp is not None and len(eng.dp.buckets) > 3
    assert (eng.dp.comm is not None) == bf16
    x, y = _batch()
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    for _ in range(3):
        if accum:
            half = per // 2
            eng.train_step([(xs[:half], ys[:half]), (xs[half:], ys[half:])])
        else:
            eng.train_step([(xs, ys)])
    flat = eng.store.master.clone()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1]), "ranks diverged"
    if rank == 0:
        torch.save(eng.model_state_dict(), os.path.join(out_dir, f"dp_{accum}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("accum,bf16", [(False, False), (True, False), (False, True)])
def test_dp_matches_single_process(tmp_path, accum, bf16):
    mp.spawn(_worker_dp, args=(2, _port(), str(tmp_path), accum, bf16), nprocs=2, join=True)
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, device=torch.device("cpu"))
    x, y = _batch()
    for _ in range(3):
        eng.train_step([(x, y)])
    dp = torch.load(tmp_path / f"dp_{accum}.pt", weights_only=True)
    for k, v in eng.model_state_dict().items():
        if bf16:
            # bf16 gradients on the wire (8 mantissa bits): Adam normalises the update, so weights
            # move by ~lr per step either way; a flipped sign on a ~0 gradient costs <= 2 lr
            assert (dp[k] - v).abs().max().item() <= 3 * 2e-2, k
            assert torch.nn.functional.cosine_similarity(dp[k].flatten() - _init_of(k),
                                                         v.flatten() - _init_of(k), dim=0) > 0.95, k
        else:
            # summation order differs (gloo sum of half-batch grads); Adam amplifies it only on ~0 grads
            torch.testing.assert_close(dp[k], v, atol=1e-4, rtol=1e-4)


def _init_of(name):
    return _model().state_dict()[name].detach().float().flatten()


class _Crossed(torch.nn.Module):
    """Registration order a, b, c but forward uses c first: the layout's reverse registration
    order (a's bucket last) is not the order gradients complete in (a's gradient first)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = torch.nn.Linear(16, 16)
        self.b = torch.nn.Linear(16, 16)
        self.c = torch.nn.Linear(16, 16)

    def forward(self, x, y):
        h = self.a(torch.tanh(self.b(torch.tanh(self.c(x)))))
        return h, ((h - y) ** 2).mean()


def _worker_relayout(rank, world, port, out_dir):
    _init(rank, world, port)
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_Crossed(), lr=1e-2, grad_clip=1.0, bucket_mb=0.0005, decay_names=set())
    before = list(eng.store.names)
    g = torch.Generator().manual_seed(rank)
    x, y = torch.randn(8, 16, generator=g), torch.randn(8, 16, generator=g)
    eng.train_step([(x, y)])
    after = list(eng.store.names)
    assert after != before and after[:2] == ["a.bias", "a.weight"] or after[:2] == ["a.weight", "a.bias"], after
    # buckets now follow the observed order: the first bucket holds only a's parameters
    first = [eng.store.names[i] for i in eng.store.buckets[0][2]]
    assert all(n.startswith("a.") for n in first), first
    for _ in range(2):
        eng.train_step([(x, y)])
    if rank == 0:
        torch.save(eng.model_state_dict(), os.path.join(out_dir, "relayout.pt"))
    import torch.distributed as dist

    dist.destroy_process_group()


def test_dp_rebuilds_buckets_in_observed_order(tmp_path):
    mp.spawn(_worker_relayout, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_Crossed(), lr=1e-2, grad_clip=1.0, device=torch.device("cpu"), decay_names=set())
    xs, ys = [], []
    for r in range(2):
        g = torch.Generator().manual_seed(r)
        xs.append(torch.randn(8, 16, generator=g))
        ys.append(torch.randn(8, 16, generator=g))
    x, y = torch.cat(xs), torch.cat(ys)
    for _ in range(3):
        eng.train_step([(x, y)])
    got = torch.load(tmp_path / "relayout.pt", weights_only=True)
    for k, v in eng.model_state_dict().items():
        torch.testing.assert_close(got[k], v, atol=1e-5, rtol=1e-5)


def _worker_trainer(rank, world, port, out_dir):
    _init(rank, world, port)
    from mingpt_distributed_amd.data import CharDataset, DataConfig
    from mingpt_distributed_amd.models import OptimizerConfig
    from mingpt_distributed_amd.optim import create_optimizer
    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import GPTTrainer, GPTTrainerConfig

    ds = CharDataset(DataConfig(block_size=16), "abcdefghijklmnopqrstuvwxyz " * 60, verbose=False)
    m = _model()
    cfg = GPTTrainerConfig(max_epochs=2, batch_size=8, grad_norm_clip=1.0, snapshot_path=os.path.join(out_dir, "s.pt"),
                           save_every=1, log_every=1000, max_steps_per_epoch=6)
    tr = GPTTrainer(cfg, m, create_optimizer(m, OptimizerConfig()), ds, None)
    assert len(tr.train_loader.sampler) == (len(ds) + 1) // 2
    tr.train()
    if rank == 0:
        assert os.path.exists(cfg.snapshot_path)
    D.destroy()


def test_gpt_trainer_two_ranks(tmp_path):
    mp.spawn(_worker_trainer, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    assert os.path.exists(tmp_path / "s.pt")


def test_torchrun_elastic_restart_resumes_from_step_snapshot(tmp_path):
    """rank 1 dies hard (os._exit) after step 7; torchrun (--max-restarts 1) restarts
    the worker group, which resumes from the step-5 snapshot and finishes the run.  c10d rendezvous
    (as ``scripts/run_node.sh`` / the reference ``slurm_run.sh:17-22`` use): a static-port restart
    can reconnect gloo to the dead group's stale addresses."""
    import subprocess
    import sys

    corpus = tmp_path / "input.txt"
    corpus.write_text("the quick brown fox jumps over the lazy dog. " * 60)
    cfg = tmp_path / "cfg.yaml"
    cfg.write_text(f"""
gpt_config: {{n_layer: 1, n_head: 2, n_embd: 32}}
optimizer_config: {{learning_rate: 0.001}}
data_config: {{path: {corpus}, block_size: 16}}
trainer_config: {{max_epochs: 1, batch_size: 8, grad_norm_clip: 1.0, snapshot_path: {tmp_path / 's.pt'},
                 save_every: 1, max_steps_per_epoch: 12, log_every: 1000, save_every_steps: 5,
                 fault_inject_step: 7, fault_inject_rank: 1, fault_inject_mode: exit}}
""")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("TORCHELASTIC_RESTART_COUNT", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--max-restarts", "1", "--rdzv-backend", "c10d", "--rdzv-endpoint", f"127.0.0.1:{_port()}",
           "-m", "mingpt_distributed_amd.train", "--config", str(cfg), "--device", "cpu"]
    r = subprocess.run(cmd, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), env=env,
                       capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "injected fault after step 7" in out
    assert "Resuming training from epoch 0 step 5" in out
    snap = torch.load(str(tmp_path / "s.pt"), weights_only=True)
    assert snap["step"] == 12 and snap["final_epoch"] == 0 and snap["epoch_step"] == 0


def _worker_comm_cpu(port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from mingpt_distributed_amd.optim import FlatParamStore
    from mingpt_distributed_amd.parallel.ddp import DataParallelEngine

    dist.init_process_group("gloo", rank=0, world_size=1)
    store = FlatParamStore(torch.nn.Linear(4, 4), device=torch.device("cpu"), bucket_numel=64)
    msgs = []
    try:
        DataParallelEngine(store, comm_at_world1=True, comm="rccl")
    except RuntimeError as e:
        msgs.append(str(e))
    try:  # the CU-sharing proxy (parallel/comm_proxy.py) models GPU collectives only
        DataParallelEngine(store, comm_at_world1=True, comm="proxy")
    except RuntimeError as e:
        msgs.append(str(e))
    eng = DataParallelEngine(store, comm_at_world1=True, comm="c10d")
    msgs.append(eng.comm_plan()["comm_backend"])
    dist.destroy_process_group()
    with open(os.path.join(out_dir, "msgs.txt"), "w") as f:
        f.write("\n".join(msgs))


def test_comm_backend_selection_cpu(tmp_path, monkeypatch):
    """The native RCCL communicator is GPU-only and says so on a CPU store; MINGPT_COMM is
    validated; c10d stays the default and is what comm_plan() reports."""
    from mingpt_distributed_amd.parallel.comm import comm_backend_default

    monkeypatch.delenv("MINGPT_COMM", raising=False)
    assert comm_backend_default() == "c10d"
    monkeypatch.setenv("MINGPT_COMM", "RCCL")
    assert comm_backend_default() == "rccl"
    monkeypatch.setenv("MINGPT_COMM", "mpi")
    with pytest.raises(ValueError):
        comm_backend_default()
    monkeypatch.delenv("MINGPT_COMM")
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker_comm_cpu, args=(_port(), str(tmp_path)))
    p.start()
    p.join(timeout=60)
    assert p.exitcode == 0
    msgs = (tmp_path / "msgs.txt").read_text().splitlines()
    assert "GPU" in msgs[0] and "GPU" in msgs[1] and msgs[2] == "c10d"


def test_comm_exit_handler_does_not_pin_communicator():
    """The communicator's atexit teardown holds it only weakly: a dropped communicator is closed
    by its own __del__ (freeing its RCCL resources then), and the exit handler skips it."""
    import gc
    import weakref

    from mingpt_distributed_amd.parallel.comm import _close_if_alive

    closed = []

    class Fake:
        def close(self):
            closed.append(1)

    f = Fake()
    ref = weakref.ref(f)
    _close_if_alive(ref)
    assert closed == [1]
    del f
    gc.collect()
    assert ref() is None
    _close_if_alive(ref)
    assert closed == [1]


def _worker_subgroup_bcast(rank, world, port, out_dir):
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.optim import FlatParamStore
    from mingpt_distributed_amd.parallel.ddp import DataParallelEngine

    sub = dist.new_group([1, 3])  # every rank creates it; only 1 and 3 use it
    if rank in (1, 3):
        torch.manual_seed(100 + rank)  # different weights per rank before the broadcast
        m = torch.nn.Linear(4, 4)
        store = FlatParamStore(m, device=torch.device("cpu"), bucket_numel=1 << 20)
        eng = DataParallelEngine(store, process_group=sub, broadcast=False)
        eng.broadcast_params(src=0)  # GROUP rank 0 = global rank 1
        torch.save(store.master.clone(), os.path.join(out_dir, f"m{rank}.pt"))
        eng.close()
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_params_src_is_a_group_rank(tmp_path):
    """DataParallelEngine.broadcast_params reads ``src`` as a rank of the engine's process group on
    both communicator paths (c10d converts it to the global rank): on the sub-group [1, 3], src 0
    is global rank 1, whose weights both members end with."""
    mp.spawn(_worker_subgroup_bcast, args=(4, _port(), str(tmp_path)), nprocs=4, join=True)
    m1 = torch.load(tmp_path / "m1.pt", weights_only=True)
    m3 = torch.load(tmp_path / "m3.pt", weights_only=True)
    torch.manual_seed(101)
    ref = torch.nn.Linear(4, 4)
    assert torch.equal(m1, m3)
    want = torch.cat([ref.weight.detach().reshape(-1), ref.bias.detach()]).sort().values
    assert torch.equal(m1[: want.numel()].sort().values, want) or torch.equal(m1[m1 != 0].sort().values, want)
