"""Parameter grouping of the overlapped optimizer (trainer.overlap_groups) and its CPU fallback."""
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.optim import FlatParamStore
from mingpt_distributed_amd.trainer import StepEngine, overlap_groups


def _model(L=3):
    torch.manual_seed(0)
    return GPT(GPTConfig(n_layer=L, n_head=2, n_embed=32, vocab_size=50, block_size=16), verbose=False)


def test_groups_cover_every_parameter_once_in_forward_order():
    m = _model()
    names = FlatParamStore(m).names
    groups, blocks = overlap_groups(m, names)
    assert len(blocks) == 3 and len(groups) == 5
    flat = [n for g in groups for n in g]
    assert sorted(flat) == sorted(names) and len(flat) == len(set(flat))
    assert set(groups[0]) == {"transformer.wte.weight", "transformer.wpe.weight"}
    for i in range(3):
        assert groups[1 + i] and all(n.startswith(f"transformer.h.{i}.") for n in groups[1 + i])
    assert all(n.startswith("transformer.ln_f.") for n in groups[4])


def test_model_without_blocks_is_one_group():
    m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 2))
    groups, blocks = overlap_groups(m, ["0.weight", "0.bias", "1.weight", "1.bias"])
    assert blocks is None and groups == [["0.weight", "0.bias", "1.weight", "1.bias"]]


def test_cpu_engine_ignores_overlap_and_still_trains():
    eng = StepEngine(_model(2), lr=1e-2, device=torch.device("cpu"), overlap_optimizer=True)
    assert not eng.overlap_optimizer
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 50, (4, 16), generator=g)
    y = torch.roll(x, -1, 1)
    l0 = eng.train_step([(x, y)]).item()
    for _ in range(5):
        l1 = eng.train_step([(x, y)]).item()
    assert l1 < l0
    assert eng.store.grad.abs().max().item() == 0.0  # zeroed after the step
