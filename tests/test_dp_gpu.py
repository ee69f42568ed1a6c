"""Data parallelism through the GPU engine: two ranks share the one card of a gpurun box.

RCCL refuses two ranks on one device, so the collectives go through ``gloo`` (CUDA tensors are
staged through host memory).  Everything else is the production path: the fused HIP ops report
parameter use / gradient readiness (``ops/grads.py``), buckets are slices of the flat fp32
main-grad buffer and launch from inside backward, ``finish()`` orders the optimizer after them.
Checks: the all-reduced gradient of a 2-rank step equals the 1-process gradient on the
concatenated batch (also with gradient accumulation), and the ranks stay bit-identical over
several optimizer steps.
"""
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from mingpt_distributed_amd.models import GPT, GPTConfig

    torch.manual_seed(0)
    return GPT(GPTConfig(n_layer=2, n_head=4, n_embed=256, vocab_size=512, block_size=128,
                         embed_drop=0.0, resid_drop=0.0, attn_drop=0.0), verbose=False)


def _batch():
    g = torch.Generator().manual_seed(1)
    return (torch.randint(0, 512, (8, 128), generator=g), torch.randint(0, 512, (8, 128), generator=g))


def _worker(rank, world, port, out_dir, accum):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist

    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    D.init_distributed(device="cuda", backend="gloo")
    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, bucket_mb=0.5, device=torch.device("cuda", 0))
    assert eng.dp is not None and len(eng.dp.buckets) > 3
    x, y = _batch()
    per = x.shape[0] // world
    xs = x[rank * per:(rank + 1) * per].cuda()
    ys = y[rank * per:(rank + 1) * per].cuda()
    # 1) the averaged gradient of one step
    if accum:
        h = per // 2
        eng.forward_backward(xs[:h], ys[:h], scale=0.5, sync=False)
        eng.forward_backward(xs[h:], ys[h:], scale=0.5, sync=True)
    else:
        eng.forward_backward(xs, ys)
    torch.cuda.synchronize()
    grad = (eng.store.grad / world).cpu()
    eng.optimizer_step()
    # 2) several optimizer steps: every rank must hold the same weights
    for _ in range(3):
        eng.train_step([(xs, ys)])
    torch.cuda.synchronize()
    torch.save({"names": list(eng.store.names), "sd": eng.model_state_dict()},
               os.path.join(out_dir, f"rank{rank}_{accum}.pt"))
    if rank == 0:
        torch.save(grad, os.path.join(out_dir, f"dp_{accum}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("accum", [False, True])
def test_gpu_dp_matches_single_process(tmp_path, accum):
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), accum)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    r0 = torch.load(tmp_path / f"rank0_{accum}.pt", weights_only=True)
    r1 = torch.load(tmp_path / f"rank1_{accum}.pt", weights_only=True)
    assert r0["names"] == r1["names"], "ranks built different bucket layouts"
    bad = [k for k in r0["sd"] if not torch.equal(r0["sd"][k], r1["sd"][k])]
    assert not bad, f"ranks diverged on {bad}"

    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=torch.device("cuda", 0))
    x, y = _batch()
    eng.forward_backward(x.cuda(), y.cuda())
    torch.cuda.synchronize()
    ref = eng.store.grad.cpu()
    dp = torch.load(tmp_path / f"dp_{accum}.pt", weights_only=True)
    # bf16 activations: half-batch and full-batch GEMM tiles round differently
    scale = ref.abs().max().item()
    torch.testing.assert_close(dp, ref, atol=2e-2 * scale, rtol=0.05)
    cos = torch.nn.functional.cosine_similarity(dp, ref, dim=0).item()
    assert cos > 0.999, cos


def _worker_zero(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist

    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    D.init_distributed(device="cuda", backend="gloo")
    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=torch.device("cuda", 0), zero1=True)
    assert eng.zero1 and eng.opt.exp_avg.numel() * world == eng.store.total
    x, y = _batch()
    per = x.shape[0] // world
    xs = x[rank * per:(rank + 1) * per].cuda()
    ys = y[rank * per:(rank + 1) * per].cuda()
    for _ in range(3):
        eng.train_step([(xs, ys)])
    eng.opt.consolidate()  # masters of the other shard, for the comparison
    eng.dp.wait_gathers()
    torch.cuda.synchronize()
    flat = eng.store.flat.detach().float().cpu()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1]), "ranks diverged"
    if rank == 0:
        torch.save(eng.model_state_dict(), os.path.join(out_dir, "zero.pt"))
    dist.destroy_process_group()


def test_gpu_zero1_matches_replicated(tmp_path):
    """ZeRO-1 through the HIP AdamW kernels on shard slices vs the replicated 1-process step."""
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_worker_zero, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]

    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=torch.device("cuda", 0))
    x, y = _batch()
    names = sorted(eng.model_state_dict())
    m0 = torch.cat([eng.model_state_dict()[k].flatten() for k in names])
    for _ in range(3):
        eng.train_step([(x.cuda(), y.cuda())])
    torch.cuda.synchronize()
    ref = torch.cat([eng.model_state_dict()[k].flatten() for k in names])
    zs = torch.load(tmp_path / "zero.pt", weights_only=True)
    z = torch.cat([zs[k].flatten() for k in names])
    # compare the parameter updates: bf16 half- vs full-batch rounding, Adam normalises it
    dz, dr = z - m0, ref - m0
    cos = torch.nn.functional.cosine_similarity(dz, dr, dim=0).item()
    assert cos > 0.99, cos
    # an Adam step moves a weight by at most ~lr, so 3 steps bound any difference by 3*lr (hit
    # only where a near-zero gradient flips sign between the two batch splits)
    diff = (z - ref).abs()
    assert diff.max().item() <= 3.5e-3, diff.max().item()
    assert (diff > 1e-4).float().mean().item() < 1e-3


# ------------------------------------------------------------------------------ RCCL paths
def _worker_rccl1(port, out_dir, zero1, bf16, comm="c10d"):
    """One rank on a real ``nccl`` (RCCL) process group with the collective path forced on:
    the bucket all-reduce / in-place reduce-scatter and all-gather calls run on RCCL (through
    c10d, or through the engine's own communicator with ``comm="rccl"``)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from mingpt_distributed_amd.trainer import StepEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=dev, bucket_mb=0.5, zero1=zero1,
                     reduce_dtype=torch.bfloat16 if bf16 else None, comm_at_world1=True, comm=comm)
    assert eng.dp is not None and eng.dp.active and len(eng.dp.buckets) > 3
    assert (eng.dp.native is not None) == (comm == "rccl")
    x, y = _batch()
    eng.measure_comm = True  # bench.py's comm_exposed_ms plumbing on the real RCCL path
    for _ in range(3):
        eng.train_step([(x.cuda(), y.cuda())])
    c = eng.comm_exposed_ms()
    assert c is not None and math.isfinite(c) and c >= 0.0, c
    plan = eng.dp.comm_plan()
    assert plan["n_buckets"] == len(eng.dp.buckets) and len(plan["bucket_bytes"]) == plan["n_buckets"]
    assert plan["wire_dtype"] == ("bf16" if bf16 else "fp32")
    assert plan["comm_backend"] == ("rccl-native" if comm == "rccl" else "c10d")
    if comm == "rccl":
        if zero1:
            eng.dp.wait_gathers()  # the parameter all-gathers are waited on by the NEXT forward
        assert eng.dp.native.pending() == 0  # every collective's ticket was waited on
    if zero1:
        eng.opt.consolidate()
        st = eng.opt.state_dict()
        assert st["step"] == 3
    torch.cuda.synchronize()
    torch.save(eng.model_state_dict(), os.path.join(out_dir, "rccl1.pt"))
    dist.destroy_process_group()


def _worker_zero1_generate(port, out_dir):
    """ZeRO-1 on a one-rank RCCL group (collective path forced): generate() right after an
    optimizer step, while the parameter all-gathers are in flight, must decode from the gathered
    weights: the same tokens as a plain copy of the trained weights."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from mingpt_distributed_amd.models import GPT
    from mingpt_distributed_amd.trainer import StepEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    model = _model()
    eng = StepEngine(model, lr=1e-3, grad_clip=1.0, device=dev, bucket_mb=0.5, zero1=True,
                     comm_at_world1=True)
    x, y = _batch()
    eng.train_step([(x.cuda(), y.cuda())])
    model.eval()
    idx = x[:1, :5].cuda()
    out = model.generate(idx, 12, do_sample=False)
    torch.cuda.synchronize()
    ref = GPT(model.config, verbose=False).to(dev).to(torch.bfloat16).eval()
    ref.load_state_dict({k: v.to(torch.bfloat16) for k, v in eng.model_state_dict().items()})
    torch.save({"out": out.cpu(), "ref": ref.generate(idx, 12, do_sample=False).cpu()},
               os.path.join(out_dir, "zgen.pt"))
    dist.destroy_process_group()


def test_gpu_zero1_generate_after_step(tmp_path):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker_zero1_generate, args=(_port(), str(tmp_path)))
    p.start()
    p.join(timeout=100)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode
    r = torch.load(tmp_path / "zgen.pt", weights_only=True)
    assert torch.equal(r["out"], r["ref"])


@pytest.mark.parametrize("comm", ["c10d", "rccl"])
@pytest.mark.parametrize("zero1,bf16", [(False, False), (False, True), (True, False), (True, True)])
def test_gpu_rccl_one_rank_collective_paths(tmp_path, zero1, bf16, comm):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker_rccl1, args=(_port(), str(tmp_path), zero1, bf16, comm))
    p.start()
    p.join(timeout=100)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode

    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=torch.device("cuda", 0))
    x, y = _batch()
    for _ in range(3):
        eng.train_step([(x.cuda(), y.cuda())])
    torch.cuda.synchronize()
    got = torch.load(tmp_path / "rccl1.pt", weights_only=True)
    init = _model().state_dict()
    du, dv = [], []
    for k, v in eng.model_state_dict().items():
        # a one-rank sum is the identity, but the wte gradient is an fp32-atomic scatter (its
        # summation order varies run to run) and bf16 on the wire rounds every gradient: Adam
        # turns either into update differences of at most ~lr per step on near-zero gradients
        # (e.g. the k-part of c_attn.bias, whose true gradient is 0)
        assert (got[k] - v).abs().max().item() <= 3.5e-3, k
        du.append((got[k] - init[k]).flatten())
        dv.append((v - init[k]).flatten())
    cos = torch.nn.functional.cosine_similarity(torch.cat(du), torch.cat(dv), dim=0).item()
    assert cos > 0.995, cos


def _worker_proxy(port, out_dir):
    """comm="proxy" (parallel/comm_proxy.py) on a one-rank group: each bucket's stand-in kernel
    runs on its own stream at the bucket-ready point, leaves the gradients alone (the weights
    match a no-communication engine's), is waited on before the optimizer, and lasts its paced
    time when alone on the GPU."""
    # 1 GB/s: the 0.5 MiB buckets of this small model last ~1 ms each, well above launch overhead
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MINGPT_PROXY_GBPS="1",
                      MINGPT_PROXY_CHANNELS="16", MINGPT_PROXY_RANKS="8")
    import torch.distributed as dist

    from mingpt_distributed_amd.trainer import StepEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=0, world_size=1)
    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=dev, bucket_mb=0.5, comm_at_world1=True,
                     comm="proxy")
    ref = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=dev)
    proxy = eng.dp.proxy
    assert proxy is not None and eng.dp.comm_plan()["comm_backend"] == "proxy" and len(eng.dp.buckets) > 3
    x, y = _batch()
    proxy.record = True
    for _ in range(3):
        eng.train_step([(x.cuda(), y.cuda())])
        ref.train_step([(x.cuda(), y.cuda())])
    assert eng.dp.proxy is proxy  # kept across the bucket relayout after step 1
    recs = proxy.take_records()
    assert recs and all(t > 0 for _, t in recs)
    a, b = eng.model_state_dict(), ref.model_state_dict()
    for k in a:  # wte's gradient is an fp32-atomic scatter: Adam may differ by ~lr there
        assert (a[k] - b[k]).abs().max().item() <= 3.5e-3, k
    iso = eng.dp.time_collectives(reps=3)
    for bk, t in zip(eng.dp.buckets, iso):
        m = proxy.model_ms((bk.end - bk.start) * 4)
        if m >= 0.2:  # (tiny buckets: launch and event overhead)
            assert 0.8 * m < t < 1.4 * m + 0.15, (t, m)
    dist.destroy_process_group()


def test_gpu_comm_proxy_one_rank(tmp_path):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker_proxy, args=(_port(), str(tmp_path)))
    p.start()
    p.join(timeout=100)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode


def _worker_nccl2(rank, world, port, out_dir, zero1, comm="c10d"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    info = D.init_distributed(device="cuda", backend="nccl")
    assert info.backend == "nccl" and dist.get_world_size() == world
    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, bucket_mb=0.5, zero1=zero1, comm=comm)
    x, y = _batch()
    per = x.shape[0] // world
    xs = x[rank * per:(rank + 1) * per].cuda()
    ys = y[rank * per:(rank + 1) * per].cuda()
    for _ in range(3):
        eng.train_step([(xs, ys)])
    if zero1:
        eng.opt.consolidate()
        eng.dp.wait_gathers()
    torch.cuda.synchronize()
    flat = eng.store.flat.detach()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert all(torch.equal(gathered[0], g) for g in gathered[1:]), "ranks diverged"
    if rank == 0:
        torch.save(eng.model_state_dict(), os.path.join(out_dir, "nccl2.pt"))
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs 2 GPUs (RCCL over xGMI)")
@pytest.mark.parametrize("comm", ["c10d", "rccl"])
@pytest.mark.parametrize("zero1", [False, True])
def test_gpu_nccl_two_gpus_match_single_process(tmp_path, zero1, comm):
    """Two ranks on two GPUs over RCCL: the N-GPU step equals the 1-process step on the
    concatenated batch, and the ranks stay bit-identical (DP all-reduce and ZeRO-1 paths; c10d's
    communicator and the engine's own)."""
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_worker_nccl2, args=(r, 2, port, str(tmp_path), zero1, comm))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]

    from mingpt_distributed_amd.trainer import StepEngine

    eng = StepEngine(_model(), lr=1e-3, grad_clip=1.0, device=torch.device("cuda", 0))
    x, y = _batch()
    for _ in range(3):
        eng.train_step([(x.cuda(), y.cuda())])
    torch.cuda.synchronize()
    got = torch.load(tmp_path / "nccl2.pt", weights_only=True)
    for k, v in eng.model_state_dict().items():
        assert (got[k] - v).abs().max().item() <= 3.5e-3, k  # half- vs full-batch bf16 rounding
