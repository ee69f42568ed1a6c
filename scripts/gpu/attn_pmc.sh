#!/bin/bash
# attention microbench (B=16/32) + two PMC passes over the B=32 fwd/bwd kernels
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-attnpmc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 200 python bench/bench_attention.py --B 32 > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d "$OUT/p1" -o a -- python3 bench/attn_pmc.py > "$OUT/p1.log" 2>&1 || { tail "$OUT/p1.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d "$OUT/p2" -o b -- python3 bench/attn_pmc.py > "$OUT/p2.log" 2>&1 || { tail "$OUT/p2.log"; exit 1; }
for f in $(find "$OUT" -name '*counter_collection.csv'); do python scripts/pmc_summary.py "$f" attn; done
