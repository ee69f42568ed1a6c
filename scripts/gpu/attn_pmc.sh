#!/bin/bash
# Attention PMC at the GPT-2 shape (B = ATTN_B, default 128; fwd p = 0.1 and 0, bwd p = 0.1):
# three counter passes, each its own run under a hard time limit.  scripts/gpu/attn_pmc.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-apmc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  ATTN_ITERS=2 timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/p$i" -o a \
    -- python3 bench/dev/attn_prof.py > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  for f in $(find "$OUT/p$i" -name '*counter_collection.csv'); do
    python scripts/pmc_summary.py "$f" attn_ > "$OUT/p$i.txt"; cat "$OUT/p$i.txt"
  done
done
