"""Comm/compute CU sharing on one GPU: the training step with a stand-in for each bucket's
N-rank all-reduce (parallel/comm_proxy.py, csrc/kernels/comm_proxy.hip) against the same step
without communication.

    python bench/comm_proxy.py --model gpt2 --batch 128 --configs 300:32:32,0:32:32,300:32:8
    python bench/comm_proxy.py --model gpt2-xl --batch 16 --configs 300:32:32

Each config is ``gbps:channels:bucket_mb[:ranks]`` (gbps 0 = unpaced copy; ranks 1 = a null
proxy: the data-parallel engine's bucket plumbing with nothing launched).  Per config, one JSON line:
step ms without communication (mean of the runs before and after), with the proxies, the
slowdown, the step's exposed-communication time (end of backward to end of the last proxy), and
per bucket its launch-to-completion time inside the step (from the moment its gradients were
ready on the device, mean over the timed steps) against its isolated time (alone on the GPU after
the timed steps) and the paced model time.  A ratio near 1 says the collectives progress beside
backward's GEMMs; well above 1 says they queue for CUs behind them.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--configs", default="300:32:32")
    a = ap.parse_args()

    from mingpt_distributed_amd.models import GPT, GPTConfig
    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    info = D.init_distributed(device="cuda", group_at_world1=True)
    dev = info.device
    V = 50257
    cfg = GPTConfig(model_type=a.model, vocab_size=V, block_size=a.seq, embed_drop=0.1, resid_drop=0.1,
                    attn_drop=0.1)
    g = torch.Generator(device=dev).manual_seed(99)
    xs = [torch.randint(0, V, (a.batch, a.seq), device=dev, generator=g) for _ in range(2)]
    ys = [torch.randint(0, V, (a.batch, a.seq), device=dev, generator=g) for _ in range(2)]

    def engine(comm, bucket_mb):
        torch.manual_seed(1234)
        m = GPT(cfg, verbose=False)
        if comm:
            return StepEngine(m, bucket_mb=bucket_mb, device=dev, comm_at_world1=True, comm="proxy")
        return StepEngine(m, device=dev)

    def timed(eng, record=False):
        for i in range(a.warmup):
            eng.train_step([(xs[i % 2], ys[i % 2])])
        torch.cuda.synchronize()
        proxy = eng.dp.proxy if eng.dp is not None else None
        if proxy is not None:
            proxy.take_records()
            proxy.record = record
            eng.measure_comm = True
            eng.comm_exposed_ms()
        t0 = time.perf_counter()
        for i in range(a.steps):
            eng.train_step([(xs[i % 2], ys[i % 2])])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps * 1e3
        recs, exposed = [], None
        if proxy is not None:
            proxy.record = False
            eng.measure_comm = False
            recs = proxy.take_records()
            exposed = eng.comm_exposed_ms()
        return dt, recs, exposed

    base = engine(False, 0)
    base_ms = [timed(base)[0]]
    print(f"# {a.model} B={a.batch}: no-comm step {base_ms[0]:.2f} ms", file=sys.stderr, flush=True)
    for spec in a.configs.split(","):
        f = spec.split(":")
        gbps, channels, bucket_mb = f[:3]
        ranks = int(f[3]) if len(f) > 3 else a.ranks
        os.environ["MINGPT_PROXY_GBPS"] = gbps
        os.environ["MINGPT_PROXY_CHANNELS"] = channels
        os.environ["MINGPT_PROXY_RANKS"] = str(ranks)
        eng = engine(True, float(bucket_mb))
        ms, recs, exposed = timed(eng, record=True)
        base_ms.append(timed(base)[0])
        proxy = eng.dp.proxy
        nb = len(eng.dp.buckets)
        per = {}  # bucket position in launch order -> in-step times
        for k, (nbytes, t) in enumerate(recs):
            per.setdefault(k % nb, []).append((nbytes, t))
        iso = eng.dp.time_collectives(reps=3)
        rows = []
        for k in range(nb):
            nbytes = per[k][0][0]
            in_step = sum(t for _, t in per[k]) / len(per[k])
            rows.append({"bucket": k, "mib": round(nbytes / 2 ** 20, 2), "in_step_ms": round(in_step, 3),
                         "isolated_ms": round(iso[k], 3), "ratio": round(in_step / max(iso[k], 1e-6), 2),
                         "model_ms": None if proxy.model_ms(nbytes) is None else round(proxy.model_ms(nbytes), 3)})
        b0 = sum(base_ms[-2:]) / 2
        out = {"model": a.model, "batch": a.batch, "ranks": ranks, "gbps": float(gbps), "channels": int(channels),
               "bucket_mb": float(bucket_mb), "n_buckets": nb, "step_ms_no_comm": round(b0, 2),
               "step_ms_proxy": round(ms, 2), "slowdown_pct": round((ms / b0 - 1) * 100, 2),
               "exposed_comm_ms": None if exposed is None else round(exposed, 3),
               "sum_isolated_ms": round(sum(iso), 2),
               "sum_in_step_ms": round(sum(r["in_step_ms"] for r in rows), 2), "buckets": rows}
        print(json.dumps(out), flush=True)
        eng.dp.close()
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
