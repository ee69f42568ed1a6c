"""AdamW step alone on a model's flat store (device time per step, median of 10 after 3 warm):
    python bench/dev/adamw_time.py --model gpt2-xl"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl")
    a = ap.parse_args()
    from mingpt_distributed_amd.models import GPT, GPTConfig
    from mingpt_distributed_amd.trainer import StepEngine

    torch.manual_seed(0)
    eng = StepEngine(GPT(GPTConfig(model_type=a.model, vocab_size=50257, block_size=1024), verbose=False),
                     device=torch.device("cuda", 0))
    eng.store.grad.normal_()
    ts = []
    for i in range(13):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        eng.opt.step(grad_scale=1.0, zero_grad=True)
        e.record()
        e.synchronize()
        if i >= 3:
            ts.append(s.elapsed_time(e))
    ts.sort()
    n = eng.store.total
    ms = ts[len(ts) // 2]
    print(json.dumps({"model": a.model, "params": n, "adamw_ms": round(ms, 3),
                      "tb_s_at_34B": round(34 * n / ms / 1e9, 2), "so": os.environ.get("MINGPT_EXT_SO", "tree")}))


if __name__ == "__main__":
    main()
