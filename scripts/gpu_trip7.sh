#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -q -p no:cacheprovider -k exact > gpurun_out/t7_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t7_tests.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dropout 0.0 > gpurun_out/t7_bench0.log 2>&1 || exit $?
