#!/bin/bash
# attention kernels (B=32, bench/attn_pmc.py): kernel stats + one PMC pass of issue/wait counters
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-attnpmc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks" -o k -- python3 bench/attn_pmc.py > "$OUT/ks.log" 2>&1 || { tail "$OUT/ks.log"; exit 1; }
python scripts/kernel_stats.py "$OUT/ks" --steps 2 | head -12
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d "$OUT/p1" -o a -- python3 bench/attn_pmc.py > "$OUT/p1.log" 2>&1 || { tail "$OUT/p1.log"; exit 1; }
for f in $(find "$OUT/p1" -name '*counter_collection.csv'); do python scripts/pmc_summary.py "$f" attn; done
