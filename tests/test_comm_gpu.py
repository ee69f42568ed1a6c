"""Native RCCL communicator (csrc/comm/rccl_comm.cpp, parallel/comm.py) on a one-rank group:
the RCCL it binds is torch's, and its collectives are ordered against the compute stream in both
directions (comm stream after the producers, consumers after wait()) without host syncs."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, path):
    import faulthandler

    faulthandler.enable()  # a crash inside RCCL / HIP prints the Python frame it happened under
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from mingpt_distributed_amd.parallel.comm import RcclCommunicator

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    c = RcclCommunicator(device=dev)
    res = {"version": c.version, "torch_version": list(torch.cuda.nccl.version())}
    n = 1 << 20
    # producer -> collective: a long spin kernel delays the fill; a comm stream that did not wait
    # for the compute stream would reduce the zeros
    for name, dt in (("f32", torch.float32), ("bf16", torch.bfloat16)):
        src = torch.zeros(n, device=dev, dtype=dt)
        out = torch.zeros(n, device=dev, dtype=dt)
        torch.cuda._sleep(50_000_000)
        src.fill_(3.0)
        w = c.reduce_scatter(src, out)
        w.wait()
        out.add_(1.0)  # collective -> consumer: must see the 3s
        g = torch.zeros(n, device=dev, dtype=dt)
        torch.cuda._sleep(50_000_000)
        out.mul_(2.0)
        c.all_gather(out, g).wait()
        buf = torch.full((n,), 5.0, device=dev, dtype=dt)
        torch.cuda._sleep(50_000_000)
        buf.add_(1.0)
        c.all_reduce(buf).wait()
        c.broadcast(buf, 0).wait()
        buf.add_(1.0)
        torch.cuda.synchronize()
        res[name] = [out.float().unique().tolist(), g.float().unique().tolist(), buf.float().unique().tolist()]
    res["pending"] = c.pending()
    try:
        c._C.comm_wait(c.handle, 10_000)
        res["bad_ticket"] = "accepted"
    except RuntimeError as e:
        res["bad_ticket"] = str(e)
    c.close()
    torch.save(res, path)
    dist.destroy_process_group()


def test_native_comm_one_rank_ordering(tmp_path):
    ctx = mp.get_context("spawn")
    out = str(tmp_path / "comm.pt")
    p = ctx.Process(target=_worker, args=(_port(), out))
    p.start()
    p.join(timeout=100)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode
    r = torch.load(out, weights_only=True)
    major, minor, patch = r["torch_version"]
    assert r["version"] == major * 10000 + minor * 100 + patch  # the RCCL torch loaded, not /opt/rocm's
    for name in ("f32", "bf16"):
        assert r[name] == [[8.0], [8.0], [7.0]], (name, r[name])  # out: (3 + 1) * 2
    assert r["pending"] == 0
    assert "ticket" in r["bad_ticket"]
