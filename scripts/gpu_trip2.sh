#!/bin/bash
mkdir -p gpurun_out
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ]; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py -q -p no:cacheprovider > gpurun_out/t2_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t2_tests.log; ok $s || exit $s
timeout -k 10 300 python bench/bench_gemm.py > gpurun_out/t2_gemm.log 2>&1 || exit $?
