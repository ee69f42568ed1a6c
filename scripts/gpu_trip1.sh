#!/bin/bash
# GPU trip 1: toolchain check (hipcc 7.2 code objects under torch's HIP 7.0 runtime),
# kernel numerics, and the torch-eager self-baseline.
mkdir -p gpurun_out
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ]; }
python -c "import torch; print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/t1_env.log 2>&1
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider > gpurun_out/t1_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t1_tests.log; ok $s || exit $s
for attn in sdpa math; do
  timeout -k 10 300 python bench/baseline_torch.py --batch 16 --steps 10 --warmup 3 --attn $attn >> gpurun_out/t1_baseline.log 2>&1 || exit $?
done
timeout -k 10 300 python bench/baseline_torch.py --batch 32 --steps 10 --warmup 3 --attn sdpa >> gpurun_out/t1_baseline.log 2>&1 || exit $?
timeout -k 10 300 python bench/baseline_torch.py --batch 16 --steps 10 --warmup 3 --attn sdpa --dropout 0.0 >> gpurun_out/t1_baseline.log 2>&1 || exit $?
