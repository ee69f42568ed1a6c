#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py -q -p no:cacheprovider > gpurun_out/t4_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t4_tests.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/t4_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/t4_bench.log 2>&1 || exit $?
