"""Per-tile phase times of attn_bwd64_kernel from a -DMG_BWD64_STAMPS build (s_memtime per wave at
8 points of each tile of the first 64 workgroups = key block 0 at the GPT-2 B = 128 shape):
    MINGPT_EXT_SO=build/ab/stamps/_C.so python bench/dev/bwd64_stamps.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from mingpt_distributed_amd.ops._ext import ext

C = ext()
C.attention_set_bwd64(1)
B, T, H, hd = int(os.environ.get("ATTN_B", "128")), 1024, 12, 64
D = H * hd
qkv = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
out, lse, mask = C.attention_fwd(qkv, B, T, H, 0.1, 1)
for _ in range(4):
    C.attention_bwd(qkv, out, dout, lse, mask, B, T, H, 0.1, 1)
torch.cuda.synchronize()
raw = C.attention_bwd64_stamps()
st = raw[:64 * 4 * 8 * 8].view(64, 4, 8, 8).double()
pe2 = raw[64 * 4 * 8 * 8:].view(64, 4, 2, 4, 2).double()  # [wg][wave][item 0 / 1][point][memtime, realtime]
pe = pe2[:, :, 0]
names = ["issue", "tile body", "barrier 1", "commit", "dQ MFMA", "dQ store", "barrier 2"]
print("phase cycles (median over workgroups and waves), tiles 0-1 diagonal, 2-7 steady")
print(f"{'tile':>4s} " + " ".join(f"{n:>10s}" for n in names) + f" {'total':>8s}")
for t in range(8):
    d = st[:, :, t, 1:] - st[:, :, t, :-1]
    med = d.reshape(-1, 7).median(0).values
    tot = (st[:, :, t, 7] - st[:, :, t, 0]).median().item()
    print(f"{t:4d} " + " ".join(f"{v:10.0f}" for v in med.tolist()) + f" {tot:8.0f}")
nxt = (st[:, :, 1:, 0] - st[:, :, :-1, 7]).median().item()
print(f"between tiles (loop overhead): {nxt:.0f}")
pro = (pe[:, :, 1, 0] - pe[:, :, 0, 0]).median().item()
loop = (pe[:, :, 2, 0] - pe[:, :, 1, 0]).median().item()
epi = (pe[:, :, 3, 0] - pe[:, :, 2, 0]).median().item()
clk = ((pe[:, :, 3, 0] - pe[:, :, 0, 0]) / (pe[:, :, 3, 1] - pe[:, :, 0, 1]) * 0.1).median().item()
wall = ((pe[:, :, 3, 1] - pe[:, :, 0, 1]) / 100).median().item()
print(f"workgroup (key block 0): prologue {pro:.0f}, tile loops {loop:.0f}, epilogue {epi:.0f} cycles; "
      f"{wall:.1f} us at {clk:.2f} GHz")
# the second work item (the workgroup's next item from the counter: its prologue is the K / V
# conversion after the first item's epilogue; its first tile and K / V were staged under it)
q = pe2[:, :, 1]
pro2 = (q[:, :, 1, 0] - q[:, :, 0, 0]).median().item()
loop2 = (q[:, :, 2, 0] - q[:, :, 1, 0]).median().item()
epi2 = (q[:, :, 3, 0] - q[:, :, 2, 0]).median().item()
print(f"second item: prologue {pro2:.0f}, tile loops {loop2:.0f}, epilogue {epi2:.0f} cycles")
