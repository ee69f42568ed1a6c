"""Model semantics on the CPU path (canonical GPT-2; reference defects D1-D10, D32 fixed)."""
import math

import pytest
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.utils import CfgNode


def _tiny(**kw):
    base = dict(n_layer=2, n_head=2, n_embed=32, vocab_size=50, block_size=16, embed_drop=0.0,
                resid_drop=0.0, attn_drop=0.0)
    base.update(kw)
    return GPT(GPTConfig(**base), verbose=False)


def test_gpt2_param_count():
    m = GPT(GPTConfig(model_type="gpt2"), verbose=False)
    assert m.num_params() == 124_439_808
    assert sum(p.numel() for p in m.parameters()) == 124_439_808  # tied lm_head
    assert m.lm_head.weight is m.transformer.wte.weight


def test_untied_param_count():
    m = GPT(GPTConfig(model_type="gpt2", tie_weights=False), verbose=False)
    assert sum(p.numel() for p in m.parameters()) == 124_439_808 + 50257 * 768


def test_canonical_names():
    names = set(dict(_tiny().named_parameters()))
    assert "transformer.h.0.attn.c_attn.weight" in names
    assert "transformer.h.1.mlp.c_proj.bias" in names
    assert "transformer.ln_f.weight" in names and "transformer.wpe.weight" in names


def test_causal_mask():
    """D4: changing token j must not change logits at positions < j."""
    torch.manual_seed(0)
    m = _tiny().eval()
    x = torch.randint(0, 50, (1, 16))
    x2 = x.clone()
    x2[0, 9] = (x2[0, 9] + 1) % 50
    l1, _ = m(x)
    l2, _ = m(x2)
    torch.testing.assert_close(l1[0, :9], l2[0, :9])
    assert not torch.allclose(l1[0, 9:], l2[0, 9:])


def test_loss_ignore_index_and_init_loss():
    torch.manual_seed(0)
    m = _tiny()
    x = torch.randint(0, 50, (4, 16))
    y = torch.randint(0, 50, (4, 16))
    _, loss = m(x, y)
    assert abs(loss.item() - math.log(50)) < 0.3
    y2 = y.clone()
    y2[:, :8] = -1
    logits, l2 = m(x, y2)
    ref = torch.nn.functional.cross_entropy(logits[:, 8:].reshape(-1, 50), y[:, 8:].reshape(-1))
    torch.testing.assert_close(l2, ref)


def test_init_statistics():
    torch.manual_seed(0)
    m = GPT(GPTConfig(n_layer=4, n_head=4, n_embed=256, vocab_size=1000, block_size=256), verbose=False)
    sd = dict(m.named_parameters())
    assert abs(sd["transformer.wpe.weight"].std().item() - 0.02) < 0.002  # D9: not zeros
    for n in ("transformer.h.0.attn.c_proj.weight", "transformer.h.0.mlp.c_proj.weight"):  # D10
        assert abs(sd[n].std().item() - 0.02 / math.sqrt(8)) < 0.001
    assert abs(sd["transformer.h.0.mlp.c_fc.weight"].std().item() - 0.02) < 0.002
    assert torch.all(sd["transformer.h.0.ln_1.weight"] == 1)


def test_block_size_enforced():
    m = _tiny()
    with pytest.raises(ValueError):
        m(torch.zeros(1, 17, dtype=torch.long))


def test_generate_kv_cache_matches_full_recompute():
    torch.manual_seed(0)
    m = _tiny().eval()
    idx = torch.randint(0, 50, (2, 5))
    a = m.generate(idx, 20, do_sample=False, use_cache=True)  # crosses block_size=16: window slides
    b = m.generate(idx, 20, do_sample=False, use_cache=False)
    assert a.shape == (2, 25)
    assert torch.equal(a, b)


def test_generate_sampling_topk():
    torch.manual_seed(0)
    m = _tiny().eval()
    idx = torch.randint(0, 50, (3, 4))
    out = m.generate(idx, 6, do_sample=True, top_k=5, temperature=0.8)
    assert out.shape == (3, 10) and torch.equal(out[:, :4], idx)


def test_upstream_cfgnode_config():
    C = GPT.get_default_config()
    C.model_type = "gpt-nano"
    C.vocab_size = 3
    C.block_size = 11
    m = GPT(C, verbose=False)
    assert m.config.n_embed == 48
    C2 = GPT.get_default_config()
    C2.model_type = None
    C2.n_layer, C2.n_head, C2.n_embd = 1, 2, 16
    C2.vocab_size, C2.block_size = 5, 8
    assert GPT(C2, verbose=False).config.n_head == 2
    C3 = GPT.get_default_config()
    C3.model_type = "gpt-nano"
    C3.n_layer, C3.n_head, C3.n_embd = 1, 2, 16
    C3.vocab_size, C3.block_size = 5, 8
    with pytest.raises(ValueError):
        GPT(C3, verbose=False)


def test_from_pretrained_synthetic_hf():
    """HF GPT2LMHeadModel -> our GPT: key mapping, Conv1D transpose, logits parity (parity
    against a randomly initialised local HF model: no real OpenAI weights are reachable)."""
    transformers = pytest.importorskip("transformers")
    torch.manual_seed(0)
    hf_cfg = transformers.GPT2Config(n_layer=2, n_head=2, n_embd=64, vocab_size=50257, n_positions=1024)
    hf = transformers.GPT2LMHeadModel(hf_cfg).eval()
    from mingpt_distributed_amd.models.pretrained import load_gpt2

    m = load_gpt2(GPT, "gpt2", source=hf, n_layer=2, n_head=2, n_embed=64).eval()
    x = torch.randint(0, 50257, (2, 12))
    with torch.no_grad():
        ref = hf(x).logits
        ours, _ = m(x)
    torch.testing.assert_close(ours, ref, atol=1e-4, rtol=1e-4)
    g1 = m.generate(x[:1, :4], 8, do_sample=False)
    g2 = hf.generate(x[:1, :4], max_new_tokens=8, do_sample=False, pad_token_id=0)
    assert torch.equal(g1, g2)


def test_gpu_shape_validation_is_early():
    """GPU-unsupported shapes are rejected on the host, before any kernel launch."""
    from mingpt_distributed_amd.models import GPTConfig

    assert GPTConfig(model_type="gpt2").resolve().gpu_unsupported() is None
    assert GPTConfig(model_type="gpt2-xl").resolve().gpu_unsupported() is None
    bad = GPTConfig(n_layer=1, n_head=3, n_embed=60).resolve()  # head dim 20, n_embed % 8 != 0
    assert "multiple of 8" in bad.gpu_unsupported()
    with pytest.raises(ValueError, match="not supported by the GPU kernels"):
        bad.check_gpu_support()


def test_gpu_head_dims_accepted():
    """Head dims the kernels take (multiples of 8 up to 128, power of two or not) pass the host
    check; 136 (> 128) and 20 (not a multiple of 8) do not."""
    from mingpt_distributed_amd.models import GPTConfig

    for hd in (8, 48, 64, 80, 96, 128):
        assert GPTConfig(n_layer=1, n_head=2, n_embed=2 * hd).resolve().gpu_unsupported() is None, hd
    assert "multiple of 8" in GPTConfig(n_layer=1, n_head=2, n_embed=272).resolve().gpu_unsupported()
    assert "multiple of 8" in GPTConfig(n_layer=1, n_head=2, n_embed=40).resolve().gpu_unsupported()
