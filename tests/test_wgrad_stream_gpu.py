"""Weight gradients on the side stream (ops/streams.py) give the gradients of the in-order
backward: one StepEngine backward of the same weights and batch with the side stream off and on,
compared on the whole flat fp32 gradient buffer (split-K fp32 atomics may add in another order,
hence a tolerance rather than bit equality), and the side stream joined by the step."""
import copy

import pytest
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.ops import streams
from mingpt_distributed_amd.trainer import StepEngine

pytestmark = pytest.mark.gpu


def _grads(base, x, y, on):
    streams.set_enabled(on, "1")  # every weight gradient on the side stream, whatever its size
    try:
        eng = StepEngine(copy.deepcopy(base), lr=1e-3)
        eng.forward_backward(x, y)
        assert not streams.pending()  # forward_backward joined the side stream
        torch.cuda.synchronize()
        return eng.store.grad.clone()
    finally:
        streams.set_enabled(True, "auto")


@pytest.mark.parametrize("n_embed,n_head", [(256, 4), (768, 12)])
def test_side_stream_grads_match_in_order(n_embed, n_head):
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=3, n_head=n_head, n_embed=n_embed, vocab_size=2048, block_size=256,
                    embed_drop=0.0, resid_drop=0.0, attn_drop=0.0)
    base = GPT(cfg, verbose=False)
    x = torch.randint(0, 2048, (8, 256), device="cuda")
    y = torch.roll(x, -1, 1)
    g0 = _grads(base, x, y, False)
    g1 = _grads(base, x, y, True)
    assert torch.isfinite(g1).all()
    torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-6 * g0.abs().max().item())


def test_side_stream_training_steps_reduce_loss():
    streams.set_enabled(True, "1")
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=2, n_head=4, n_embed=256, vocab_size=1000, block_size=128,
                    embed_drop=0.1, resid_drop=0.1, attn_drop=0.1)
    eng = StepEngine(GPT(cfg, verbose=False), lr=1e-3)
    x = torch.randint(0, 1000, (8, 128), device="cuda")
    y = torch.roll(x, -1, 1)
    try:
        losses = [eng.train_step([(x, y)]).item() for _ in range(20)]
    finally:
        streams.set_enabled(True, "auto")
    assert losses[-1] < losses[0] - 1.0, losses


def test_auto_mode_picks_small_weight_gradients():
    streams.set_enabled(True, "auto")
    assert streams.use_for(16384) and not streams.use_for(32768) and not streams.use_for(131072)


def _ws_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ws_worker(port, path, comm):
    """One-rank RCCL group (comm_at_world1): the gradient buckets' all-reduces are issued while
    block weight gradients are still pending on the side stream (ddp.py launches them on the
    collective stream after those), with the fp32 and the bf16 wire, side stream off and on."""
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=3, n_head=4, n_embed=256, vocab_size=2048, block_size=256,
                    embed_drop=0.0, resid_drop=0.0, attn_drop=0.0)
    base = GPT(cfg, verbose=False)
    x = torch.randint(0, 2048, (8, 256), device="cuda")
    y = torch.roll(x, -1, 1)
    res = {}
    for wire in ("fp32", "bf16"):
        for on in (False, True):
            streams.set_enabled(on, "1")
            try:
                eng = StepEngine(copy.deepcopy(base), lr=1e-3, bucket_mb=0.25, comm_at_world1=True, comm=comm,
                                 reduce_dtype=torch.bfloat16 if wire == "bf16" else None)
                assert eng.dp is not None and eng.dp.active and len(eng.dp.buckets) > 3
                eng.forward_backward(x, y)
                assert not streams.pending()
                g = eng.dp.grad_buffer.float().clone()
                eng.optimizer_step()
                torch.cuda.synchronize()
                res[(wire, on)] = (g.cpu(), eng.store.master.clone().cpu())
                native = eng.dp.native
                eng.dp.close()
                if native is not None:
                    native.close()
            finally:
                streams.set_enabled(True, "auto")
    torch.save({f"{w}_{int(o)}": v for (w, o), v in res.items()}, path)
    dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["c10d", "rccl"])
def test_side_stream_with_collectives_at_world1(tmp_path, comm):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    out = str(tmp_path / "ws.pt")
    p = ctx.Process(target=_ws_worker, args=(_ws_port(), out, comm))
    p.start()
    p.join(timeout=150)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode
    r = torch.load(out, weights_only=True)
    for wire in ("fp32", "bf16"):
        g0, w0 = r[f"{wire}_0"]
        g1, w1 = r[f"{wire}_1"]
        assert torch.isfinite(g1).all() and torch.isfinite(w1).all()
        tol = 1e-6 if wire == "fp32" else 1e-2  # bf16 wire: rounding of slightly different sums
        torch.testing.assert_close(g1, g0, rtol=1e-3 if wire == "bf16" else 1e-4,
                                   atol=tol * g0.abs().max().item())
        torch.testing.assert_close(w1, w0, rtol=1e-4, atol=1e-5)
