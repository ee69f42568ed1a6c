#!/bin/bash
mkdir -p gpurun_out
for b in 16 32; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/t10_bench_b$b.log 2>&1 || exit $?
done
timeout -k 10 300 python bench/baseline_torch.py --batch 32 --steps 10 --warmup 3 --attn sdpa > gpurun_out/t10_base32.log 2>&1 || exit $?
