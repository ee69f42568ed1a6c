#!/bin/bash
mkdir -p gpurun_out/prof2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof2/bench.log 2>&1 || exit $?
