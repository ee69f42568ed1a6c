import sys, os, torch
sys.path.insert(0, os.getcwd())
from mingpt_distributed_amd.models import GPT, GPTConfig
torch.manual_seed(0)
m = GPT(GPTConfig(model_type="gpt2", vocab_size=50257, block_size=1024), verbose=False).cuda().to(torch.bfloat16).eval()
idx = torch.randint(0, 50257, (1, 32), device="cuda")
with torch.no_grad():
    m.generate(idx, 8, do_sample=False)
    torch.cuda.synchronize()
    m.generate(idx, 64, do_sample=False)
    torch.cuda.synchronize()
