import sys, os
sys.path.insert(0, os.getcwd())
import torch
from mingpt_distributed_amd.ops._ext import ext
C = ext()
B, T, H, hd = 64, 1024, 12, 64
D = H * hd
qkv = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
out, lse, mask = C.attention_fwd(qkv, B, T, H, 0.1, 1)
for mode in (1, 2, 1, 2):
    C.attention_set_bwd_mode(mode)
    for _ in range(2): C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, 0.1, 1)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, 0.1, 1)
    e.record(); torch.cuda.synchronize()
    print("mode", mode, round(s.elapsed_time(e) / 10, 3), "ms")
