#!/bin/bash
# per-kernel time of the flagship bench step (kernel trace + stats only; no PMC)
mkdir -p gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof1/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1b -o run -- python3 bench/baseline_torch.py --batch 16 --steps 5 --warmup 2 --attn sdpa > gpurun_out/prof1/baseline.log 2>&1 || exit $?
ls -R gpurun_out/prof1 gpurun_out/prof1b | head -30
