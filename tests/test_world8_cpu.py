"""Eight ranks over gloo on CPU: the world size of one MI355X node (BASELINE configs #3 and #5).

The same engine code drives RCCL on the GPUs; the paths that only a wide world exercises are
checked here (the 2-rank tests in test_distributed_cpu.py / test_zero_cpu.py cannot see them):

* DP with fp32 and bf16 gradients on the wire: the 8-rank step equals the 1-process step on the
  concatenated batch (bf16: within the rounding of 8 summed bf16 contributions), and all ranks
  hold bit-identical weights after 3 steps.  The model ties ``wte`` / ``lm_head`` and the tied
  weight is bigger than a bucket, so it travels alone in its own bucket (``FlatParamStore``).
* The observed-order bucket re-layout after step 1, decided once on rank 0 and broadcast.
* ZeRO-1: buckets padded to ``world * 64`` elements, interleaved shards, 8 reduce-scatter /
  all-gather participants; equality with the 1-process step, consolidate + replicated resume.

Reference: the DDP wrap ``/root/reference/mingpt/trainer.py:71`` and its sampler ``:73-81``.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

from test_distributed_cpu import _Crossed, _init, _port

WORLD = 8


def _model():
    from mingpt_distributed_amd.models import GPT, GPTConfig

    torch.manual_seed(0)
    # wte (256 x 32 = 8192 floats) > the 0.01 MiB (2621-float) bucket: it gets a bucket of its own
    return GPT(GPTConfig(n_layer=2, n_head=2, n_embed=32, vocab_size=256, block_size=16, embed_drop=0.0,
                         resid_drop=0.0, attn_drop=0.0), verbose=False)


def _batch():
    g = torch.Generator().manual_seed(1)
    return (torch.randint(0, 256, (2 * WORLD, 16), generator=g),
            torch.randint(0, 256, (2 * WORLD, 16), generator=g))


def _shard(t, rank):
    per = t.shape[0] // WORLD
    return t[rank * per:(rank + 1) * per]


def _same_everywhere(flat):
    import torch.distributed as dist

    gathered = [torch.empty_like(flat) for _ in range(dist.get_world_size())]
    dist.all_gather(gathered, flat)
    return all(torch.equal(gathered[0], g) for g in gathered[1:])


def _worker_dp(rank, world, port, out_dir, bf16):
    torch.set_num_threads(1)
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, bucket_mb=0.01,
                     reduce_dtype=torch.bfloat16 if bf16 else None)
    st = eng.store
    wte = st.index[id(eng.model.transformer.wte.weight)]
    alone = [b for b in st.buckets if wte in b[2]]
    assert len(alone) == 1 and alone[0][2] == [wte], "the tied wte must travel in its own bucket"
    assert len(eng.dp.buckets) > 4
    x, y = _batch()
    for _ in range(3):
        eng.train_step([(_shard(x, rank), _shard(y, rank))])
    assert _same_everywhere(eng.store.master.clone()), "ranks diverged"
    plan = eng.dp.comm_plan()
    assert plan["wire_dtype"] == ("bf16" if bf16 else "fp32") and plan["n_buckets"] == len(eng.dp.buckets)
    if rank == 0:
        torch.save({"model": eng.model_state_dict(), "norm": eng.grad_norm.clone()},
                   os.path.join(out_dir, f"dp8_{bf16}.pt"))
    dist.destroy_process_group()


def _single_process(steps=3):
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, device=torch.device("cpu"))
    x, y = _batch()
    for _ in range(steps):
        eng.train_step([(x, y)])
    return eng


@pytest.mark.parametrize("bf16", [False, True])
def test_dp_world8_matches_single_process(tmp_path, bf16):
    mp.spawn(_worker_dp, args=(WORLD, _port(), str(tmp_path), bf16), nprocs=WORLD, join=True)
    eng = _single_process()
    got = torch.load(tmp_path / f"dp8_{bf16}.pt", weights_only=True)
    init = _model().state_dict()
    for k, v in eng.model_state_dict().items():
        if bf16:
            # each rank's gradient is rounded to bf16 before the sum and the ring rounds the
            # partial sums again: Adam turns that into update differences of at most ~lr per
            # step, only where a gradient is near 0 (its sign can flip)
            assert (got["model"][k] - v).abs().max().item() <= 3 * 1e-2 + 1e-6, k
            d_got, d_ref = got["model"][k].flatten() - init[k].flatten(), v.flatten() - init[k].flatten()
            assert torch.nn.functional.cosine_similarity(d_got, d_ref, dim=0) > 0.95, k
        else:
            torch.testing.assert_close(got["model"][k], v, atol=1e-4, rtol=1e-4)
    if not bf16:
        torch.testing.assert_close(got["norm"], eng.grad_norm, atol=1e-5, rtol=1e-4)


def _worker_relayout(rank, world, port, out_dir):
    torch.set_num_threads(1)
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_Crossed(), lr=1e-2, grad_clip=1.0, bucket_mb=0.0005, decay_names=set())
    before = list(eng.store.names)
    g = torch.Generator().manual_seed(rank)
    x, y = torch.randn(2, 16, generator=g), torch.randn(2, 16, generator=g)
    eng.train_step([(x, y)])
    after = list(eng.store.names)
    assert after != before and set(after[:2]) == {"a.weight", "a.bias"}, after
    # every rank adopted the same layout (rank 0's decision, broadcast)
    names = [None] * world
    dist.all_gather_object(names, after)
    assert all(n == names[0] for n in names)
    for _ in range(2):
        eng.train_step([(x, y)])
    assert _same_everywhere(eng.store.master.clone())
    if rank == 0:
        torch.save(eng.model_state_dict(), os.path.join(out_dir, "relayout8.pt"))
    dist.destroy_process_group()


def test_relayout_world8(tmp_path):
    mp.spawn(_worker_relayout, args=(WORLD, _port(), str(tmp_path)), nprocs=WORLD, join=True)
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_Crossed(), lr=1e-2, grad_clip=1.0, device=torch.device("cpu"), decay_names=set())
    xs, ys = [], []
    for r in range(WORLD):
        g = torch.Generator().manual_seed(r)
        xs.append(torch.randn(2, 16, generator=g))
        ys.append(torch.randn(2, 16, generator=g))
    x, y = torch.cat(xs), torch.cat(ys)
    for _ in range(3):
        eng.train_step([(x, y)])
    got = torch.load(tmp_path / "relayout8.pt", weights_only=True)
    for k, v in eng.model_state_dict().items():
        torch.testing.assert_close(got[k], v, atol=1e-5, rtol=1e-5)


def _worker_zero(rank, world, port, out_dir, bf16):
    torch.set_num_threads(1)
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.parallel.zero import ZeroAdamW
    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, zero1=True, bucket_mb=0.01,
                     reduce_dtype=torch.bfloat16 if bf16 else None)
    assert isinstance(eng.opt, ZeroAdamW)
    for s, e, _ in eng.store.buckets:
        assert (e - s) % (world * 64) == 0, "ZeRO-1 buckets are padded to world * 64"
    own = eng.dp.own
    assert all(hi - lo == (b.end - b.start) // world for (lo, hi), b in zip(own, eng.dp.buckets))
    assert eng.opt.exp_avg.numel() * world == eng.store.total
    x, y = _batch()
    for _ in range(3):
        eng.train_step([(_shard(x, rank), _shard(y, rank))])
    eng.opt.consolidate()
    assert _same_everywhere(eng.store.master.clone()), "ranks diverged"
    if rank == 0:
        torch.save({"model": eng.model_state_dict(), "opt": eng.opt.state_dict()},
                   os.path.join(out_dir, f"zero8_{bf16}.pt"))
    dist.destroy_process_group()


def _worker_zero_resume(rank, world, port, out_dir):
    torch.set_num_threads(1)
    _init(rank, world, port)
    import torch.distributed as dist

    from mingpt_distributed_amd.trainer import StepEngine

    sd = torch.load(os.path.join(out_dir, "zero8_False.pt"), weights_only=True)
    eng = StepEngine(_model(), lr=1e-2, grad_clip=1.0, zero1=True, bucket_mb=0.01)
    eng.load_model_state_dict(sd["model"])
    eng.opt.load_state_dict(sd["opt"])
    x, y = _batch()
    eng.train_step([(_shard(x, rank), _shard(y, rank))])
    eng.opt.consolidate()
    if rank == 0:
        torch.save(eng.model_state_dict(), os.path.join(out_dir, "zero8_resumed.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("bf16", [False, True])
def test_zero1_world8_matches_single_process_and_resumes(tmp_path, bf16):
    mp.spawn(_worker_zero, args=(WORLD, _port(), str(tmp_path), bf16), nprocs=WORLD, join=True)
    eng = _single_process()
    z = torch.load(tmp_path / f"zero8_{bf16}.pt", weights_only=True)
    for k, v in eng.model_state_dict().items():
        tol = 3e-2 + 1e-6 if bf16 else 1e-4
        assert (z["model"][k] - v).abs().max().item() <= tol, k
    ref = eng.opt.state_dict()
    if not bf16:
        for name, ent in ref["state"].items():
            torch.testing.assert_close(z["opt"]["state"][name]["exp_avg"], ent["exp_avg"], atol=1e-4, rtol=1e-4)
        # consolidated state -> 8 fresh sharded ranks -> one more step == the 1-process 4th step
        mp.spawn(_worker_zero_resume, args=(WORLD, _port(), str(tmp_path)), nprocs=WORLD, join=True)
        x, y = _batch()
        eng.train_step([(x, y)])
        resumed = torch.load(tmp_path / "zero8_resumed.pt", weights_only=True)
        for k, v in eng.model_state_dict().items():
            torch.testing.assert_close(resumed[k], v, atol=1e-4, rtol=1e-4)
