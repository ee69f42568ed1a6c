"""bench.py's multi-rank fail-fast and self-check fields, on CPU gloo ranks.

The driver's N-GPU run (``python -m torch.distributed.run ... bench.py --gpus N``) must end with a
diagnosis rather than a bare timeout: a rank stuck in a phase exits non-zero within
``--phase-timeout``, naming the phase and the gradient collectives that have not completed
(bench.py ``PhaseWatchdog``).  The reference's only parallelism is DDP over NCCL
(/root/reference/mingpt/trainer.py:71, launched one rank per GPU by
/root/reference/mingpt/slurm/slurm_run.sh:17-23).
"""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--model", "gpt-nano", "--seq", "64", "--batch", "4", "--vocab", "65",
         "--steps", "3", "--warmup", "2", "--also-batch", "0"]


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.update(env_extra or {})
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return r, time.monotonic() - t0


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("extra_args", [[], ["--zero1"], ["--reduce-dtype", "bf16"]])
def test_two_ranks_report_identical_replicas_and_collective_times(extra_args):
    r, _ = _run(["--gpus", "2", *SMALL, *extra_args])
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_line(r.stdout)
    c = j["comm"]
    assert j["n_gpus"] == 2 and c["world_size"] == 2
    assert c["ranks_identical"] is True
    assert len(c["bucket_collective_ms"]) == c["n_buckets"] == len(c["bucket_busbw_gbs"])
    assert all(t > 0 for t in c["bucket_collective_ms"])
    want = "bf16" if "bf16" in extra_args else "fp32"  # fp32 unless asked: the reference's DDP wire
    assert j["config"]["grad_reduce_dtype"] == want and c["wire_dtype"] == want
    nc = j["extra"]["no_comm"]
    if "--zero1" in extra_args:
        assert nc is None  # the sharded update needs the reduce-scatter
    else:
        assert nc["ms_per_step"] > 0 and nc["value"] > 0
        assert "exposed_comm_ms_per_step" in nc


def test_one_rank_reports_null_multi_rank_fields():
    r, _ = _run(["--gpus", "1", *SMALL])
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_line(r.stdout)
    assert j["extra"]["no_comm"] is None
    c = j["comm"]
    for k in ("ranks_identical", "bucket_collective_ms", "bucket_busbw_gbs", "collective_total_ms",
              "comm_exposed_ms"):
        assert c[k] is None, (k, c[k])


@pytest.mark.parametrize("phase", ["timed step 1", "broadcast"])
def test_stalled_rank_fails_fast_naming_the_phase(phase):
    limit = 8
    r, dt = _run(["--gpus", "2", *SMALL, "--phase-timeout", str(limit)],
                 env_extra={"MINGPT_BENCH_STALL": f"1:{phase}"})
    assert r.returncode != 0
    assert dt < 6 * limit + 60, dt  # well inside the driver's 600 s, not the pg timeout
    err = r.stderr
    assert f"phase '{phase}' exceeded {limit} s" in err, err[-3000:]
    if phase.startswith("timed"):
        # the healthy rank names the bucket whose all-reduce never completed
        assert "incomplete gradient collectives (bucket, elements): [(0," in err, err[-3000:]
