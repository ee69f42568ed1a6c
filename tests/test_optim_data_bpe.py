"""Optimizer grouping/flat store/fused AdamW (CPU path), datasets, samplers, BPE."""
import copy
import json

import pytest
import torch

from mingpt_distributed_amd.bpe import BPETokenizer, Encoder, bytes_to_unicode, get_encoder
from mingpt_distributed_amd.data import AdditionDataset, CharDataset, DataConfig, SortDataset, SyntheticTokens
from mingpt_distributed_amd.models import GPT, GPTConfig, OptimizerConfig
from mingpt_distributed_amd.optim import FlatParamStore, FusedAdamW, create_optimizer, param_groups
from mingpt_distributed_amd.parallel.sampler import DistributedSampler, InfiniteRandomSampler


def _tiny():
    return GPT(GPTConfig(n_layer=2, n_head=2, n_embed=32, vocab_size=50, block_size=16, embed_drop=0.0,
                         resid_drop=0.0, attn_drop=0.0), verbose=False)


# ------------------------------------------------------------------ optimizer
def test_param_groups():
    m = _tiny()
    decay, no_decay = param_groups(m)
    assert "transformer.h.0.attn.c_attn.weight" in decay
    assert "transformer.h.0.mlp.c_fc.bias" in no_decay
    assert "transformer.wte.weight" in no_decay and "transformer.ln_f.weight" in no_decay
    assert not decay & no_decay and decay | no_decay == set(dict(m.named_parameters()))
    opt = create_optimizer(m, OptimizerConfig())
    assert [g["weight_decay"] for g in opt.param_groups] == [0.1, 0.0]
    assert opt.param_groups[0]["betas"] == (0.9, 0.95)


def test_flat_store_views_and_alignment():
    m = _tiny()
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    s = FlatParamStore(m)
    for n, p in m.named_parameters():
        torch.testing.assert_close(p.detach(), before[n])
        assert p.main_grad.shape == p.shape and p.main_grad.data_ptr() >= s.grad.data_ptr()
    assert all(o % 64 == 0 for o in s.offsets)
    assert s.names[-1] == "transformer.wte.weight"  # completes last in backward: last bucket


def test_fused_adamw_cpu_matches_torch():
    torch.manual_seed(0)
    m = _tiny()
    ref = copy.deepcopy(m)
    decay, _ = param_groups(m)
    s = FlatParamStore(m)
    opt = FusedAdamW(s, lr=1e-3, weight_decay=0.1, decay_names=decay, grad_clip=0.5)
    ropt = create_optimizer(ref, OptimizerConfig(learning_rate=1e-3))
    x = torch.randint(0, 50, (2, 16))
    for _ in range(3):
        for model in (m, ref):
            _, loss = model(x, x)
            loss.backward()
        for p in m.parameters():
            p.main_grad.copy_(p.grad)
            p.grad = None
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
        ropt.step()
        ropt.zero_grad()
        opt.step()
        s.zero_grad()
    for (n, p), (_, r) in zip(m.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.detach(), r.detach(), atol=1e-5, rtol=1e-4, msg=n)
    sd = opt.state_dict()
    opt2 = FusedAdamW(FlatParamStore(copy.deepcopy(m)), decay_names=decay)
    opt2.load_state_dict(sd)
    assert opt2.step_count == 3
    torch.testing.assert_close(opt2.exp_avg, opt.exp_avg)


# ------------------------------------------------------------------ data
def test_char_dataset_fsspec_memory():
    import fsspec

    with fsspec.open("memory://corpus.txt", "w") as f:
        f.write("hello world! " * 50)
    ds = CharDataset(DataConfig(path="memory://corpus.txt", block_size=8, truncate=0.5), verbose=False)
    assert ds.vocab_size == len(set("hello world! "))
    assert len(ds) == len("hello world! " * 50) // 2 - 8
    x, y = ds[3]
    assert x.dtype == torch.long and torch.equal(x[1:], y[:-1])
    assert ds.decode(ds.encode("hello")) == "hello"
    ds2 = CharDataset(DataConfig(block_size=4), "abcabc", verbose=False)  # upstream (config, data) form
    assert ds2.get_vocab_size() == 3 and ds2.get_block_size() == 4


def test_sort_dataset():
    ds = SortDataset("train", length=6, num_digits=3)
    x, y = ds[0]
    assert x.shape == (11,) and y.shape == (11,)
    assert (y[:5] == -1).all()
    inp = x[:6]
    assert torch.equal(torch.cat([x[6:], y[-1:]]), torch.sort(inp)[0])
    test = SortDataset("test")
    assert all(ds._split_of(ds[i][0][:6]) == "train" for i in range(20))
    assert all(test._split_of(test[i][0][:6]) == "test" for i in range(20))


def test_addition_dataset():
    ds = AdditionDataset("train", ndigit=2)
    assert len(ds) + len(AdditionDataset("test", ndigit=2)) == 10000
    x, y = ds[0]
    digits = torch.cat([x, y[-1:]]).tolist()
    a = digits[0] * 10 + digits[1]
    b = digits[2] * 10 + digits[3]
    c = int("".join(map(str, digits[4:][::-1])))
    assert a + b == c and (y[:3] == -1).all()


def test_synthetic_tokens_deterministic():
    ds = SyntheticTokens(vocab_size=100, block_size=8, size=10)
    assert torch.equal(ds[3][0], ds[3][0]) and ds[3][0].max() < 100


def test_distributed_sampler_set_epoch_and_shards():
    data = list(range(10))
    s0 = DistributedSampler(data, num_replicas=2, rank=0)
    s1 = DistributedSampler(data, num_replicas=2, rank=1)
    e0 = list(s0)
    s0.set_epoch(1)
    assert list(s0) != e0  # D20: reshuffled every epoch
    s1.set_epoch(1)
    assert sorted(list(s0) + list(s1)) == data
    it = iter(InfiniteRandomSampler(data, rank=1))
    assert all(0 <= next(it) < 10 for _ in range(100))


# ------------------------------------------------------------------ BPE
def _toy_encoder(tmp_path):
    """A synthetic byte-level BPE: all 256 byte symbols + a few merges (no OpenAI files here)."""
    b2u = bytes_to_unicode()
    vocab = {c: i for i, c in enumerate(b2u.values())}
    merges = [("h", "e"), ("l", "l"), ("he", "ll"), ("Ġ", "w"), ("o", "r")]
    for a, b in merges:
        vocab[a + b] = len(vocab)
    (tmp_path / "encoder.json").write_text(json.dumps(vocab))
    (tmp_path / "vocab.bpe").write_text("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n")
    return vocab


def test_bpe_roundtrip_and_merges(tmp_path):
    vocab = _toy_encoder(tmp_path)
    enc = get_encoder(str(tmp_path))
    ids = enc.encode("hello world")
    assert vocab["hell"] in ids and vocab["Ġw"] in ids and vocab["or"] in ids
    assert enc.decode(ids) == "hello world"
    text = "Ünïcödé ✓ 123 'll it's\n\ttabs"
    assert enc.decode(enc.encode(text)) == text
    tok = BPETokenizer(directory=str(tmp_path))
    t = tok("hello")
    assert t.shape[0] == 1 and tok.decode(t[0]) == "hello"


def test_bpe_missing_files(tmp_path):
    with pytest.raises(FileNotFoundError):
        get_encoder(str(tmp_path / "nope"))


def test_bucket_plan_tied_embedding_alone():
    """FlatParamStore's bucket cut: a parameter at least a bucket large gets a bucket of its own
    (GPT-2's tied wte, ready only after the embedding backward, does not hold back the smaller
    gradients before it); buckets are contiguous, cover every parameter once, and a ZeRO-style
    bucket_align pads each bucket to a multiple of it."""
    from mingpt_distributed_amd.models import GPT, GPTConfig
    from mingpt_distributed_amd.optim import FlatParamStore

    m = GPT(GPTConfig(n_layer=2, n_head=2, n_embed=64, vocab_size=4096, block_size=64), verbose=False)
    cap = 4096 * 64  # = numel(wte)
    for align in (64, 4 * 64):
        st = FlatParamStore(m, device="cpu", bucket_numel=cap, bucket_align=align)
        seen = []
        prev_end = 0
        for s, e, ps in st.buckets:
            assert s == prev_end and (e - s) % align == 0
            prev_end = e
            seen += ps
            for i in ps:
                assert s <= st.offsets[i] and st.offsets[i] + st.numels[i] <= e
        assert sorted(seen) == list(range(len(st.params))) and prev_end == st.total
        wte = st.by_name["transformer.wte.weight"]
        (b,) = [ps for _, _, ps in st.buckets if wte in ps]
        assert b == [wte]


def test_fused_adamw_cpu_zero_grad_flag():
    m = torch.nn.Linear(4, 3)
    s = FlatParamStore(m)
    opt = FusedAdamW(s, lr=1e-2)
    s.grad.normal_()
    opt.step(zero_grad=True)
    assert s.grad.abs().max().item() == 0.0
