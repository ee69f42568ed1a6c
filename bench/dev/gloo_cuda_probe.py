#!/usr/bin/env python
"""Probe: gloo's in-place reduce_scatter_tensor / all_gather_into_tensor on CUDA tensors (two ranks
on one GPU, the tests/test_dp_gpu.py setting).  One JSON line per rank."""
import json
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(r, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=r, world_size=2)
    res = {"rank": r}
    n, sh = 2048, 1024
    for dt in (torch.float32, torch.bfloat16):
        try:
            wire = (torch.arange(n, device="cuda") % 5).to(dt) * (r + 1)
            out = wire[r * sh:(r + 1) * sh]
            dist.reduce_scatter_tensor(out, wire, async_op=True).wait()
            exp = ((torch.arange(n, device="cuda") % 5).to(dt) * 3)[r * sh:(r + 1) * sh]
            res[f"rs_{dt}"] = bool(torch.equal(out, exp))
        except Exception as e:  # noqa: BLE001
            res[f"rs_{dt}"] = repr(e)[:200]
        try:
            full = torch.zeros(n, device="cuda", dtype=dt)
            full[r * sh:(r + 1) * sh] = r + 1
            dist.all_gather_into_tensor(full, full[r * sh:(r + 1) * sh], async_op=True).wait()
            res[f"ag_{dt}"] = bool(torch.equal(full.float().cpu(), torch.tensor([1.0, 2.0]).repeat_interleave(sh)))
        except Exception as e:  # noqa: BLE001
            res[f"ag_{dt}"] = repr(e)[:200]
    q.put(res)
    dist.destroy_process_group()


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=90)
        if p.is_alive():
            p.kill()
    while not q.empty():
        print(json.dumps(q.get()))
