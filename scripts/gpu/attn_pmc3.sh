#!/bin/bash
# attention backward PMC at the bench shape (B=64), persistent vs partial schedule
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-apmc3}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for M in 1 2; do
  ATTN_B=64 ATTN_BWD_MODE=$M timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/m$M" -o a -- python3 bench/attn_pmc.py > "$OUT/m$M.log" 2>&1 || { tail "$OUT/m$M.log"; exit 1; }
  echo "== mode $M"; for f in $(find "$OUT/m$M" -name '*counter_collection.csv'); do python scripts/pmc_summary.py "$f" attn_bwd_kernel; done
done
