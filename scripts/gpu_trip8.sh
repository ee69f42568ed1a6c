#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/ -m gpu -q -p no:cacheprovider > gpurun_out/t8_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t8_tests.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 300 python bench/bench_gemm.py > gpurun_out/t8_gemm.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/t8_bench.log 2>&1 || exit $?
timeout -k 10 120 build/bin/xgmi_probe > gpurun_out/t8_xgmi.log 2>&1 || exit $?
