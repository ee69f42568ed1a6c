#!/bin/bash
mkdir -p gpurun_out/prof3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof3/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench/bench_attention.py > gpurun_out/prof3/attention_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench/bench_gemm.py > gpurun_out/prof3/gemm_bench.log 2>&1 || exit $?
