"""ZeRO-1 (optimizer-state sharding, parallel/zero.py) on CPU over gloo: the sharded step equals
the 1-process step on the concatenated batch, ranks agree bit for bit, each rank holds only its
shard of the Adam moments, and consolidate() + state_dict() round-trips through a replicated
optimizer's load_state_dict."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from test_distributed_cpu import _batch, _init, _model, _port


def _worker_zero(rank, world, port, out_dir, accum):
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.parallel.zero import ZeroAdamW
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, zero1=True, bucket_mb=0.01)
    assert eng.zero1 and isinstance(eng.opt, ZeroAdamW)
    assert len(eng.dp.buckets) > 3  # one reduce-scatter / all-gather per bucket
    assert eng.opt.exp_avg.numel() * world == eng.store.total
    x, y = _batch()
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    for _ in range(3):
        if accum:
            half = per // 2
            eng.train_step([(xs[:half], ys[:half]), (xs[half:], ys[half:])])
        else:
            eng.train_step([(xs, ys)])
    eng.opt.consolidate()
    flat = eng.store.master.clone()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    for g in gathered[1:]:
        assert torch.equal(gathered[0], g), "ranks diverged"
    if rank == 0:
        sd = eng.opt.state_dict()
        with pytest.raises(RuntimeError):  # the host copy is dropped once read
            eng.opt.state_dict()
        torch.save({"model": eng.model_state_dict(), "opt": sd, "norm": eng.grad_norm.clone()},
                   os.path.join(out_dir, f"zero_{accum}.pt"))
    else:
        with pytest.raises(RuntimeError):  # only rank 0 assembles the full state
            eng.opt.state_dict()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,accum", [(2, False), (2, True), (4, False)])
def test_zero1_matches_single_process(tmp_path, world, accum):
    mp.spawn(_worker_zero, args=(world, _port(), str(tmp_path), accum), nprocs=world, join=True)
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, device=torch.device("cpu"))
    x, y = _batch()
    for _ in range(3):
        eng.train_step([(x, y)])
    z = torch.load(tmp_path / f"zero_{accum}.pt", weights_only=True)
    ref_sd = eng.model_state_dict()
    for k, v in ref_sd.items():  # by name: the ZeRO layout pads every bucket
        torch.testing.assert_close(z["model"][k], v, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(z["norm"], eng.grad_norm, atol=1e-4, rtol=1e-4)
    # the consolidated ZeRO state loads into the replicated optimizer and matches its moments
    ref = eng.opt.state_dict()
    for name, ent in ref["state"].items():
        torch.testing.assert_close(z["opt"]["state"][name]["exp_avg"], ent["exp_avg"], atol=1e-4, rtol=1e-4)
    eng.opt.load_state_dict(z["opt"])
    assert eng.opt.step_count == 3


def _worker_resume(rank, world, port, out_dir):
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.trainer import StepEngine

    sd = torch.load(os.path.join(out_dir, "ref.pt"), weights_only=True)
    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, zero1=True)
    eng.load_model_state_dict(sd["model"])
    eng.opt.load_state_dict(sd["opt"])
    x, y = _batch()
    per = x.shape[0] // world
    eng.train_step([(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])])
    eng.opt.consolidate()
    if rank == 0:
        torch.save(eng.model_state_dict(), os.path.join(out_dir, "resumed.pt"))
    dist.destroy_process_group()


def test_zero1_resumes_from_replicated_snapshot(tmp_path):
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, device=torch.device("cpu"))
    x, y = _batch()
    for _ in range(2):
        eng.train_step([(x, y)])
    torch.save({"model": eng.model_state_dict(), "opt": eng.opt.state_dict()}, tmp_path / "ref.pt")
    eng.train_step([(x, y)])
    mp.spawn(_worker_resume, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    resumed = torch.load(tmp_path / "resumed.pt", weights_only=True)
    for k, v in eng.model_state_dict().items():
        torch.testing.assert_close(resumed[k], v, atol=1e-4, rtol=1e-4)


def _worker_trainer_zero(rank, world, port, out_dir):
    _init(rank, world, port)
    from mingpt_distributed_amd.data import CharDataset, DataConfig
    from mingpt_distributed_amd.models import OptimizerConfig
    from mingpt_distributed_amd.optim import create_optimizer
    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import GPTTrainer, GPTTrainerConfig

    ds = CharDataset(DataConfig(block_size=16), "abcdefghijklmnopqrstuvwxyz " * 60, verbose=False)
    m = _model()
    cfg = GPTTrainerConfig(max_epochs=2, batch_size=8, grad_norm_clip=1.0, save_every=1, log_every=1000,
                           snapshot_path=os.path.join(out_dir, "s.pt"), max_steps_per_epoch=4, zero1=True)
    tr = GPTTrainer(cfg, m, create_optimizer(m, OptimizerConfig()), ds, None)
    assert tr.engine.zero1
    tr.train()
    D.destroy()


def test_gpt_trainer_zero1_snapshot(tmp_path):
    """Sharded optimizer state is consolidated on every rank before rank 0 writes the snapshot."""
    mp.spawn(_worker_trainer_zero, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    snap = torch.load(tmp_path / "s.pt", weights_only=True)
    st = snap["optimizer_state"]
    assert st["step"] == 8 and all(e["exp_avg"].abs().sum() > 0 for e in st["state"].values())
