"""Bench-scale parity: the GPT-2 124M width (D = 768, H = 12, V = 50257, T = 1024) at a batch
large enough that the bench step's GEMM tile picks are taken (W4 forward / data-gradient tiles,
split-K weight gradients, the LM head's 128x96 data-gradient tile) compared with the fp32
PyTorch reference model on the same bf16-rounded weights (one forward + backward).
Reference semantics: ``/root/reference/mingpt/model.py:309-320`` (loss with ignore_index=-1)."""
import copy

import pytest
import torch

from mingpt_distributed_amd.models import GPT, GPTConfig

pytestmark = pytest.mark.gpu

B, T = 9, 1024  # M = 9216 tokens


@pytest.fixture(scope="module")
def reference():
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=2, n_head=12, n_embed=768, vocab_size=50257, block_size=T, embed_drop=0.0,
                    resid_drop=0.0, attn_drop=0.0)
    cpu = GPT(cfg, verbose=False)
    with torch.no_grad():  # the reference computes in fp32 on the bf16-rounded weights
        for p in cpu.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 50257, (B, T), generator=g)
    y = torch.randint(0, 50257, (B, T), generator=g)
    y[0, :7] = -1
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    logits, loss = cpu(x, y)
    loss.backward()
    rows = torch.arange(0, B * T, 97)  # a strided sample of logit rows (the full fp32 set is 1.9 GB)
    ref = {"loss": loss.item(), "logits": logits.detach().reshape(B * T, -1)[rows].clone(), "rows": rows,
           "grads": {n: p.grad.clone() for n, p in cpu.named_parameters()}}
    del logits
    cpu.zero_grad(set_to_none=True)
    return cpu, x, y, ref


def test_gpt2_width_fwd_bwd_matches_fp32(reference):
    cpu, x, y, ref = reference
    M = B * T
    gpu = copy.deepcopy(cpu).cuda().to(torch.bfloat16)
    logits, loss = gpu(x.cuda(), y.cuda())
    assert abs(loss.item() - ref["loss"]) < 1e-2, (loss.item(), ref["loss"])
    got = logits.reshape(M, -1)[ref["rows"].cuda()].float().cpu()
    torch.testing.assert_close(got, ref["logits"], atol=5e-2, rtol=5e-2)
    del logits
    loss.backward()
    for n, p in gpu.named_parameters():
        gc, gg = ref["grads"][n], p.grad.float().cpu()
        scale = gc.abs().max().item() + 1e-12
        err = (gg - gc).abs().max().item() / scale
        cos = torch.nn.functional.cosine_similarity(gg.flatten(), gc.flatten(), dim=0).item()
        assert err < 0.05 and cos > 0.999, f"{n}: max rel err {err:.4f}, cos {cos:.5f}"
