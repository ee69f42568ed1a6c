#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gemm_gpu.py -q -p no:cacheprovider -x > gpurun_out/t9_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t9_tests.log
[ $s -eq 0 ] || exit $s
timeout -k 10 300 python bench/bench_gemm.py > gpurun_out/t9_gemm.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/t9_bench.log 2>&1 || exit $?
