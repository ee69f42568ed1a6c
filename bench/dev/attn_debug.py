"""Forward attention vs fp32 reference over head dims / dropout (debug aid)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_attention_gpu import _dense_keep, _split
from mingpt_distributed_amd.ops._ext import ext
C = ext()
DEV = "cuda"
for hd in [8, 16, 24, 32, 64]:
    for T in [200, 128, 64]:
        B, H = 2, 2
        torch.manual_seed(hd)
        D = H * hd
        qkv = torch.randn(B * T, 3 * D, device=DEV).to(torch.bfloat16)
        q, k, v = _split(qkv, B, T, H)
        att = (q @ k.transpose(-1, -2)) / hd ** 0.5
        att = att.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=DEV).tril(), float("-inf"))
        for p in (0.0, 0.1):
            out, lse, mask = C.attention_fwd(qkv, B, T, H, p, 5)
            keep = _dense_keep(mask, B, T, H) * (256.0 / (256 - round(p * 256))) if p > 0 else 1.0
            ref = ((att.softmax(-1) * keep) @ v).transpose(1, 2).reshape(B * T, D)
            err = (out.float() - ref).abs()
            bad = (err > 3e-2 + 3e-2 * ref.abs())
            lse_ref = torch.logsumexp(att, -1) / torch.log(torch.tensor(2.0))
            lerr = (lse.view(B, H, T) - lse_ref).abs().max().item()
            rows = bad.any(1).nonzero().flatten().tolist()
            print(f"hd {hd} T {T} p {p}: max err {err.max().item():.4f} bad {bad.sum().item()} lse err {lerr:.4f} rows {rows[:12]}")
