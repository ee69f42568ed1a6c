#!/bin/bash
# one PMC pass over both attention backward kernels (MINGPT_ATTN_BWD4=1 / 0)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-b4pmc}; mkdir -p "$OUT"; export TMPDIR=/tmp
P="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
for v in 1 0; do
  i=0
  for PP in "$P" "$P2"; do
    i=$((i + 1))
    MINGPT_ATTN_BWD4=$v ATTN_ITERS=2 timeout -s KILL 90 rocprofv3 --pmc $PP --kernel-trace --output-format csv -d "$OUT/v$v$i" -o a \
      -- python3 bench/dev/attn_prof.py > "$OUT/v$v$i.log" 2>&1 || { echo "pass failed"; tail -5 "$OUT/v$v$i.log"; exit 1; }
    for f in $(find "$OUT/v$v$i" -name '*counter_collection.csv'); do
      python scripts/pmc_summary.py "$f" attn_bwd > "$OUT/v$v$i.txt"; cat "$OUT/v$v$i.txt"
    done
  done
done
