"""Attention kernels at the bench shape for rocprofv3 kernel stats (fwd p=0.1 / p=0, bwd p=0.1)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from mingpt_distributed_amd.ops._ext import ext
C = ext()
B, T, H, hd = int(os.environ.get("ATTN_B", "128")), 1024, 12, 64
D = H * hd
qkv = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
for _ in range(int(os.environ.get("ATTN_ITERS", "5"))):
    out, lse, mask = C.attention_fwd(qkv, B, T, H, 0.1, 1)
    C.attention_fwd(qkv, B, T, H, 0.0, 1)
    if os.environ.get("ATTN_BWD", "1") == "1":
        C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, 0.1, 1)
torch.cuda.synchronize()
print("done")
