#!/usr/bin/env python
"""Flagship benchmark: GPT-2 124M, seq 1024, bf16 training throughput (tokens/s, whole node).

Metric/config are the ones BASELINE.json names.  One process per GPU (torchrun env), data
parallel over RCCL.  Synthetic random-token batches of the exact training shape and random-init
weights (no datasets or checkpoints are reachable); every timed step is a full training step:
forward, backward, bucketed all-reduce, global grad-norm clip and fused AdamW update, with the
reference's dropout (0.1) active.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model gpt2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

``--gpus N > 1`` without a torchrun env starts the N ranks itself (a child
``torch.distributed.run``); a rank whose process group is not N wide exits non-zero instead of
reporting a smaller run under the requested GPU count.

W untimed warmup steps, then K steps bracketed by barrier + device sync; the max over ranks is
reported.  The same engine is then timed again at ``--also-batch`` sequences per GPU (default 64,
the reference's per-GPU batch, ``/root/reference/mingpt/gpt2_config.yaml:14``), reported under
``extra`` so that rounds stay comparable at a fixed config.

Diagnostics in the JSON line (``comm``): the RCCL version the ranks loaded, every rank's device
name and PCI bus id, the bucket plan (count, bytes per bucket in the wire dtype), and
``comm_exposed_ms`` -- the mean device time per timed step from the end of backward's last
kernel to the end of the gradient communication (``StepEngine.comm_exposed_ms``): the
communication NOT hidden under backward.  ``--comm-at-world1`` runs the RCCL path on a one-rank
group at N = 1 as a plumbing check of those fields.  ``vs_baseline`` divides by N x the measured single-GPU torch-eager self-baseline of the
same step at the same per-GPU batch, i.e. the per-GPU speedup over stock
PyTorch-ROCm (the reference publishes no numbers).

Gradient wire dtype: fp32 by default, the reference DDP's precision
(``/root/reference/mingpt/trainer.py:71``); ``--reduce-dtype bf16`` is a labelled variant
(``config.grad_reduce_dtype``).  At N > 1 a compute-only pass follows the checksum: the same
steps with every gradient collective skipped (``StepEngine.train_step_local``), reported as
``extra.no_comm`` (null at N = 1 and under ZeRO-1), so a 1 -> N loss splits into exposed
communication vs compute slowed by the collective kernels sharing the CUs.

Fail-fast for N > 1 (the driver's multi-GPU run must end with a diagnosis, not a bare timeout):
every rank runs a phase watchdog (:class:`PhaseWatchdog`): init, broadcast, every warmup and
timed step (one phase each), checksum, collective timing, barrier.  A phase that lasts more than ``--phase-timeout`` seconds
(default 150) prints the rank, the phase, how long it has been stuck and the gradient buckets
whose collective has not completed on the device, then exits the rank with status 4 (the
launcher then stops the others).  The process group's own timeout (``--pg-timeout``, default
180 s, RCCL async error handling on) is the backstop.  After the timed loop every rank's fp64
checksum of its weights is all-gathered: ``comm.ranks_identical`` (null at N = 1).  Per-bucket
collective time and bus bandwidth, measured in isolation after training, sit next to
``comm_exposed_ms`` (``comm.bucket_collective_ms`` / ``bucket_busbw_gbs``; null at N = 1).
``MINGPT_BENCH_STALL=rank:phase`` makes that rank hang at that phase (the fail-fast test).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch

# single-GPU torch-eager self-baseline at the SAME per-GPU batch, model, shape and dropout
# (bench/baseline_torch.py: torch.autocast bf16, SDPA attention, torch AdamW, MI355X):
# BASELINE.md "Self-baseline" table.
BASELINE_TOK_S_PER_GPU = {16: 367595.5, 32: 413092.9, 64: 461947.8, 128: 470388.8}


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


EXIT_HANG = 4


class PhaseWatchdog:
    """Names the phase a rank is in; exits the rank (status 4) when one phase outlives
    ``limit_s``, printing the phase and the gradient collectives still incomplete on the device.
    A daemon thread polling twice a second: a rank blocked inside a collective, a device sync or
    a barrier cannot report anything itself.  ``os._exit`` (no exec, no cleanup that could block
    on the hung collective)."""

    def __init__(self, rank: int, limit_s: float, engine_ref=lambda: None):
        self.rank, self.limit = rank, float(limit_s)
        self.engine_ref = engine_ref
        self.name, self.t0 = "start", time.monotonic()
        self.cur_limit = self.limit
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._stall = os.environ.get("MINGPT_BENCH_STALL", "")
        self._th = threading.Thread(target=self._run, name="bench-phase-watchdog", daemon=True)
        if self.limit > 0:
            self._th.start()

    def phase(self, name: str, limit_s: float = None):
        """Enter phase ``name`` (its own limit if given: the rendezvous waits for every rank's
        first ``import torch``, which takes minutes on a cold box)."""
        with self._lock:
            self.name, self.t0 = name, time.monotonic()
            self.cur_limit = self.limit if limit_s is None else float(limit_s)
        if self._stall and self._stall == f"{self.rank}:{name}":  # fault injection (tests)
            print(f"bench.py[rank {self.rank}]: MINGPT_BENCH_STALL: hanging in phase '{name}'",
                  file=sys.stderr, flush=True)
            while True:
                time.sleep(3600)

    def stop(self):
        """Stop and join the thread (a daemon thread still polling at interpreter shutdown is
        torn down mid-wait, which aborts the process)."""
        self._stop.set()
        if self._th.is_alive():
            self._th.join(timeout=5)

    def _run(self):
        while not self._stop.wait(0.5):
            with self._lock:
                name, el, lim = self.name, time.monotonic() - self.t0, self.cur_limit
            if el <= lim:
                continue
            msg = f"bench.py[rank {self.rank}]: phase '{name}' exceeded {lim:.0f} s ({el:.0f} s)"
            try:
                eng = self.engine_ref()
                dp = getattr(eng, "dp", None)
                if dp is not None and hasattr(dp, "incomplete_collectives"):
                    bad = dp.incomplete_collectives()
                    msg += (f"; incomplete gradient collectives (bucket, elements): {bad}" if bad
                            else "; every gradient collective of the last step completed")
            except Exception as e:  # noqa: BLE001 -- diagnostics only
                msg += f"; (collective state unavailable: {e})"
            # a grace period before exiting: the first rank to exit makes torchrun SIGTERM the
            # others, whose own watchdogs (same limit, phases entered within a poll or two) would
            # otherwise be killed before printing their diagnosis -- usually the informative one
            # (the healthy rank blocked in the collective names the bucket)
            grace = min(10.0, max(3.0, 0.25 * lim))
            print(msg + f" -- exiting in {grace:.0f} s", file=sys.stderr, flush=True)
            if self._stop.wait(grace):  # the run finished meanwhile: stop() joins this thread
                return
            os._exit(EXIT_HANG)


def _launch_ranks(n: int, device: str = "cuda") -> int:
    """``--gpus N`` without a torchrun env: start N rank processes (one per GPU) as a CHILD
    ``torch.distributed.run`` and return its exit code.  Runs before anything touches the GPU
    (``torch.cuda.device_count()`` does not initialise HIP on this image); never execs."""
    have = torch.cuda.device_count() if device == "cuda" else n
    if have < n:
        print(f"bench.py: --gpus {n} requested but only {have} GPU(s) are visible", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    print(f"bench.py: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def _ranks_identical(eng, N):
    """Collective.  fp64 checksums of this rank's weights -- the bf16 compute weights every rank
    holds in full (ZeRO-1 included) and, when replicated, the fp32 masters -- all-gathered:
    True when every rank's are bitwise equal (DP keeps the replicas identical), None at N = 1."""
    import torch.distributed as dist

    if N <= 1 or not dist.is_initialized():
        return None
    s = eng.store
    bufs = [s.flat] + ([s.master] if (s.master is not s.flat and not eng.zero1) else [])
    sums = []
    for b in bufs:
        x = b.detach().reshape(-1)
        sums += [x.sum(dtype=torch.float64), x.double().square().sum(), x[::7].sum(dtype=torch.float64)]
    mine = torch.stack(sums)
    allr = [torch.empty_like(mine) for _ in range(N)]
    dist.all_gather(allr, mine)
    return bool(all(torch.equal(allr[0], t) for t in allr[1:]))


def _collective_timing(eng, N):
    """Collective.  Isolated time and bus bandwidth of every gradient bucket's collective, in
    launch order (after the timed steps; DataParallelEngine.time_collectives)."""
    if N <= 1 or eng.dp is None or not eng.dp.active:
        return {"bucket_collective_ms": None, "bucket_busbw_gbs": None, "collective_total_ms": None}
    from mingpt_distributed_amd.parallel import dist as D

    ms = eng.dp.time_collectives()
    ms = [D.all_reduce_max(x, eng.device) for x in ms]
    bw = [eng.dp.bus_bytes(b) / (t * 1e-3) / 1e9 if t > 0 else None for b, t in zip(eng.dp.buckets, ms)]
    return {"bucket_collective_ms": [round(x, 4) for x in ms],
            "bucket_busbw_gbs": [None if x is None else round(x, 1) for x in bw],
            "collective_total_ms": round(sum(ms), 3)}


def _comm_diag(eng, info, N, comm_ms, cuda=True):
    """Self-diagnosis of the data-parallel path (collective: every rank calls it)."""
    import torch.distributed as dist

    rccl = None
    if cuda:
        try:
            v = torch.cuda.nccl.version()
            rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001 - diagnostics only
            rccl = None
    bus = None
    if cuda:
        props = torch.cuda.get_device_properties(info.device)
        bus = "%04x:%02x:%02x" % (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", 0),
                                  getattr(props, "pci_device_id", 0))
    me = {"rank": info.rank, "local_rank": info.local_rank,
          "device": torch.cuda.get_device_name(info.device) if cuda else "cpu",
          "pci_bus_id": bus, "hostname": socket.gethostname()}
    ranks = [me]
    if dist.is_initialized() and dist.get_world_size() > 1:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, me)
    out = {"rccl_version": rccl, "world_size": N, "backend": info.backend, "ranks": ranks,
           "comm_exposed_ms": None if comm_ms is None else round(comm_ms, 3)}
    if eng.dp is not None:
        out.update(eng.dp.comm_plan())
        if eng.dp.native is not None:
            out["rccl_version_native"] = eng.dp.native.version_str
    else:
        out.update({"n_buckets": None, "bucket_bytes": None, "wire_dtype": None, "collective": None,
                    "comm_backend": None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128,
                    help="sequences per GPU per step (128 x 1024 tokens: ~66 GB of the 288 GB HBM; "
                         "B = 64 / 96 / 128 measured 989.7k / 998.1k / 1,009.4k tok/s on one box, "
                         "profiles/round2_s8_batch_sweep.txt)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--vocab", type=int, default=50257, help="65 = chargpt's character vocabulary")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--reduce-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="gradient dtype on the wire for N > 1: fp32 (default, the reference DDP's "
                         "precision) or bf16 (half the xGMI bytes; reported as a labelled variant)")
    ap.add_argument("--no-comm-pass", type=int, default=1,
                    help="N > 1: after the checksum, time the same steps with every gradient "
                         "collective skipped (dp.no_sync): extra.no_comm (0: skip)")
    ap.add_argument("--zero1", action="store_true",
                    help="shard the AdamW state over the ranks (reduce-scatter + all-gather)")
    ap.add_argument("--profile", default="", help="write a torch.profiler trace to this dir")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as one hipGraph (single GPU; StepEngine.graph_step)")
    ap.add_argument("--also-batch", type=int, default=64,
                    help="second timed pass at this per-GPU batch (0: skip), reported under 'extra'")
    ap.add_argument("--comm-at-world1", action="store_true",
                    help="N = 1: drive the RCCL collective path on a one-rank group (plumbing check)")
    ap.add_argument("--comm", default=None, choices=["c10d", "rccl"],
                    help="gradient communicator: c10d's RCCL process group (default, or MINGPT_COMM) "
                         "or the engine's own RCCL communicator + comm stream (parallel/comm.py)")
    ap.add_argument("--phase-timeout", type=float, default=150.0,
                    help="N > 1: exit a rank (status 4) whose phase lasts longer, naming it (0: off)")
    ap.add_argument("--pg-timeout", type=int, default=180,
                    help="process-group collective timeout in seconds (backstop of --phase-timeout)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo ranks on the host (tests of the multi-rank plumbing only)")
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(a.gpus, a.device))  # parent: no GPU call happens in this process

    from mingpt_distributed_amd.models import GPT, GPTConfig
    from mingpt_distributed_amd.parallel import dist as D
    from mingpt_distributed_amd.trainer import StepEngine

    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")  # a timed-out collective aborts
    env_rank = int(os.environ.get("RANK", "0"))
    eng_box = []
    wd = PhaseWatchdog(env_rank, a.phase_timeout if a.gpus > 1 else 0.0,
                       engine_ref=lambda: eng_box[0] if eng_box else None)
    cuda = a.device == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda *args: None)
    wd.phase("init (rendezvous, process group)", limit_s=2 * a.phase_timeout)
    info = D.init_distributed(device=a.device, group_at_world1=a.comm_at_world1, timeout_s=a.pg_timeout)
    N = D.world_size()  # from the process group itself, not the env
    if N != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the process group has {N} rank(s); refusing to "
              f"report a {N}-GPU number as a {a.gpus}-GPU one", file=sys.stderr)
        sys.exit(3)
    dev_name = torch.cuda.get_device_name(info.device) if cuda else "cpu"
    print(f"[rank {info.rank}/{N}] local_rank {info.local_rank} on {dev_name} "
          f"({info.device}), backend {info.backend}", file=sys.stderr, flush=True)
    torch.manual_seed(1234 + info.rank)
    cfg = GPTConfig(model_type=a.model, vocab_size=a.vocab, block_size=a.seq, embed_drop=a.dropout,
                    resid_drop=a.dropout, attn_drop=a.dropout)
    torch.manual_seed(1234)  # identical init on every rank (the engine also broadcasts rank 0)
    model = GPT(cfg, verbose=info.rank == 0)
    wd.phase("broadcast")  # engine construction: rank 0's weights broadcast to every rank
    eng = StepEngine(model, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, grad_clip=1.0,
                     bucket_mb=a.bucket_mb, zero1=a.zero1, device=info.device,
                     reduce_dtype=torch.bfloat16 if a.reduce_dtype == "bf16" else None,
                     comm_at_world1=a.comm_at_world1, comm=a.comm)
    eng_box.append(eng)
    g = torch.Generator(device=eng.device).manual_seed(99 + info.rank)
    step = (lambda x, y: eng.graph_step(x, y)) if a.graph else (lambda x, y: eng.train_step([(x, y)]))

    def timed(batch, steps, warmup, profile="", tag="", step_fn=step):
        """W untimed steps, then `steps` timed ones between barrier + device syncs; returns
        (max seconds over ranks, last loss, mean exposed-comm ms or None)."""
        nb = 4
        xs = [torch.randint(0, a.vocab, (batch, a.seq), device=eng.device, generator=g) for _ in range(nb)]
        ys = [torch.randint(0, a.vocab, (batch, a.seq), device=eng.device, generator=g) for _ in range(nb)]
        for i in range(warmup):
            wd.phase(f"warmup{tag} step {i}")
            loss = step_fn(xs[i % nb], ys[i % nb])
            if i == 0:
                sync()  # the first step (bucket relayout broadcast included) completes here
        wd.phase(f"barrier before timed{tag}")
        D.barrier()
        sync()
        eng.measure_comm = eng.dp is not None and not a.graph and cuda and step_fn is step
        eng.comm_exposed_ms()  # drop warm-up events
        wd.phase(f"timed{tag} step 0")
        prof = None
        if profile and info.rank == 0:
            prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                      torch.profiler.ProfilerActivity.CUDA])
            prof.__enter__()
        t0 = time.perf_counter()
        for i in range(steps):
            if i:  # one phase per step: a long healthy run is never mistaken for a hang
                wd.phase(f"timed{tag} step {i}")
            loss = step_fn(xs[i % nb], ys[i % nb])
        wd.phase(f"timed{tag} device sync")
        sync()
        wd.phase(f"barrier after timed{tag}")
        D.barrier()
        dt = time.perf_counter() - t0
        eng.measure_comm = False
        if prof is not None:
            prof.__exit__(None, None, None)
            os.makedirs(profile, exist_ok=True)
            prof.export_chrome_trace(os.path.join(profile, "trace.json"))
            with open(os.path.join(profile, "summary.txt"), "w") as f:
                f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
        comm = eng.comm_exposed_ms()
        wd.phase(f"max over ranks{tag}")
        if comm is not None:
            comm = D.all_reduce_max(comm, eng.device)
        return D.all_reduce_max(dt, eng.device), loss, comm

    dt, loss, comm_ms = timed(a.batch, a.steps, a.warmup, a.profile)
    loss_v = D.all_reduce_mean(loss.float()).item()
    tokens = a.batch * a.seq * a.steps * N
    value = tokens / dt
    max_mem = torch.cuda.max_memory_allocated() / 2 ** 30 if cuda else None
    extra = {}
    if a.also_batch and a.also_batch != a.batch:
        dt2, _, comm2 = timed(a.also_batch, a.steps, min(a.warmup, 2), tag=f" batch{a.also_batch}")
        v2 = a.also_batch * a.seq * a.steps * N / dt2
        base2 = BASELINE_TOK_S_PER_GPU.get(a.also_batch)
        extra[f"batch{a.also_batch}"] = {
            "value": round(v2, 1), "ms_per_step": round(dt2 / a.steps * 1e3, 3),
            "global_batch": a.also_batch * N, "comm_exposed_ms": None if comm2 is None else round(comm2, 3),
            "vs_baseline": round(v2 / (base2 * N), 3) if base2 and a.model == "gpt2" and a.seq == 1024 else None}
    wd.phase("checksum")
    if eng.zero1 and eng.dp is not None:
        eng.dp.wait_gathers()  # the last step's parameter all-gathers are still in flight
    sync()
    identical = _ranks_identical(eng, N)
    wd.phase("collective timing")
    coll = _collective_timing(eng, N)
    # compute-only pass: the same steps with no gradient collective, so the 1 -> N loss splits
    # into exposed communication (ms_per_step - no_comm) and compute slowed by sharing the node
    # (no_comm vs the N = 1 step).  Replicas diverge from here on: it runs after the checksum.
    extra["no_comm"] = None
    if N > 1 and a.no_comm_pass and eng.dp is not None and not eng.zero1:
        local = lambda x, y: eng.train_step_local([(x, y)])  # noqa: E731
        dt3, _, _ = timed(a.batch, a.steps, min(a.warmup, 2), tag=" no_comm", step_fn=local)
        extra["no_comm"] = {"value": round(a.batch * a.seq * a.steps * N / dt3, 1),
                            "ms_per_step": round(dt3 / a.steps * 1e3, 3),
                            "exposed_comm_ms_per_step": round((dt - dt3) / a.steps * 1e3, 3)}
    wd.phase("report")
    diag = _comm_diag(eng, info, N, comm_ms, cuda)
    diag["ranks_identical"] = identical
    diag.update(coll)
    if info.rank == 0:
        out = {
            "metric": "tokens/sec (whole node), GPT-2 124M seq1024 bf16" if a.model == "gpt2"
            else f"tokens/sec (whole node), {a.model} seq{a.seq} vocab{a.vocab} bf16",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (BASELINE_TOK_S_PER_GPU[a.batch] * N), 3)
            if a.model == "gpt2" and a.seq == 1024 and a.vocab == 50257 and a.batch in BASELINE_TOK_S_PER_GPU
            else None,
            "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)",
            "config": {"model": a.model, "global_batch": a.batch * N, "seq_len": a.seq,
                       "parallelism": f"dp{N}" + ("-zero1" if eng.zero1 else ""), "micro_batch_per_gpu": a.batch, "dropout": a.dropout,
                       "bucket_mb": a.bucket_mb, "grad_reduce_dtype": a.reduce_dtype if N > 1 else None,
                       "hip_graph": bool(a.graph and N == 1)},
            "loss": round(loss_v, 4),
            "max_mem_gb": None if max_mem is None else round(max_mem, 2),
            "extra": extra,
            "comm": diag,
        }
        print(json.dumps(out), flush=True)
    wd.phase("destroy")
    D.destroy()
    wd.stop()


if __name__ == "__main__":
    main()
