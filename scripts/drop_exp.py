import sys, torch
sys.path.insert(0, '.')
from mingpt_distributed_amd.models import GPT, GPTConfig
from mingpt_distributed_amd.trainer import StepEngine
for ad, rd in [(0.0, 0.0), (0.1, 0.0), (0.0, 0.1), (0.1, 0.1)]:
    torch.manual_seed(0)
    m = GPT(GPTConfig(model_type='gpt2', block_size=1024, attn_drop=ad, resid_drop=rd, embed_drop=rd), verbose=False)
    e = StepEngine(m)
    g = torch.Generator(device='cuda').manual_seed(5)
    x = torch.randint(0, 50257, (4, 1024), device='cuda', generator=g)
    y = torch.randint(0, 50257, (4, 1024), device='cuda', generator=g)
    ls = [e.train_step([(x, y)]).item() for _ in range(25)]
    print(f"attn_drop={ad} resid_drop={rd}: " + " ".join(f"{v:.3f}" for v in ls[::3]), flush=True)
