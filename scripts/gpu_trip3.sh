#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_attention_gpu.py -q -p no:cacheprovider -x > gpurun_out/t3_tests.log 2>&1
s=$?; echo "pytest exit $s" >> gpurun_out/t3_tests.log; exit $s
