#!/usr/bin/env python
"""Probe: can two RCCL ranks share one GPU (a 1-GPU box)?  Two spawned processes on cuda:0,
init_process_group("nccl", world_size=2), one all_reduce and one reduce_scatter_tensor.  Prints one
JSON line per rank, or the error RCCL raises."""
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", 0))
        x = torch.full((1024,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        y = torch.empty(512, device="cuda")
        dist.reduce_scatter_tensor(y, torch.arange(1024, device="cuda", dtype=torch.float32))
        torch.cuda.synchronize()
        q.put({"rank": rank, "all_reduce": x[0].item(), "reduce_scatter_first": y[0].item()})
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put({"rank": rank, "error": repr(e)[:400]})


if __name__ == "__main__":
    import socket

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
    print(json.dumps({"exitcodes": [p.exitcode for p in ps]}))
    sys.exit(0)
