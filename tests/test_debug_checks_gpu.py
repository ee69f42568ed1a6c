"""Debug build: ``build/debug/_C.so`` (-DMG_DEBUG) under ``MINGPT_DEBUG_CHECKS=1``.

A token id or target outside the vocabulary would read (embedding fwd, cross-entropy) or
atomically write (embedding bwd) out of bounds in the release kernels.  The debug kernels clamp the
index, set a device error bit, and the checked extension proxy raises ``DeviceCheckError`` naming
the op -- no GPU fault.  Runs in a child process: one process holds one build of the extension.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

CHILD = r'''
import torch
from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.ops._ext import DeviceCheckError, ext
from mingpt_distributed_amd.trainer import StepEngine

C = ext()
assert C.debug_build(), "expected the MG_DEBUG build"
torch.manual_seed(0)
V = 512
cfg = GPTConfig(n_layer=1, n_head=2, n_embed=128, vocab_size=V, block_size=64)
eng = StepEngine(GPT(cfg, verbose=False), device=torch.device("cuda", 0))
x = torch.randint(0, V, (2, 64), device="cuda")
y = torch.randint(0, V, (2, 64), device="cuda")
l0 = eng.train_step([(x, y)]).item()  # valid ids: no check fires
assert l0 == l0
for what, xb, yb in (("embedding_fwd", x.clone().index_fill_(1, torch.tensor([5], device="cuda"), V), y),
                     ("cross-entropy", x, y.clone().index_fill_(1, torch.tensor([7], device="cuda"), V + 3))):
    try:
        eng.train_step([(xb, yb)])
    except DeviceCheckError as e:
        assert what in str(e), str(e)
        print("caught:", e)
    else:
        raise AssertionError(f"{what}: out-of-range index not reported")
    eng.store.zero_grad()
    assert C.debug_error_bits() == 0
print("debug checks ok")
'''


def test_debug_build_reports_out_of_range_indices():
    so = os.path.join(ROOT, "build", "debug", "_C.so")
    assert os.path.exists(so), "build/debug/_C.so missing: python build_ext.py --debug"
    env = dict(os.environ, MINGPT_EXT_SO=so, MINGPT_DEBUG_CHECKS="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "debug checks ok" in r.stdout
    assert r.stdout.count("caught:") == 2
