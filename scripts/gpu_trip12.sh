#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/ -m gpu -q -p no:cacheprovider -x > gpurun_out/t12_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t12_tests.log
[ $s -eq 0 ] || exit $s
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/t12_bench.log 2>&1 || exit $?
