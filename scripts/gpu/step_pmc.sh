#!/bin/bash
# Whole-step PMC of the flagship bench (B = 128, 1 timed + 1 warmup step, no B = 64 pass): two
# counter passes, each its own run under a hard time limit; stops at the first failed pass.
#   scripts/gpu/step_pmc.sh TAG      -> gpurun_out/TAG/p{1,2}.txt (per-kernel, per-dispatch sums)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-spmc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/p$i" -o s \
    -- python3 bench.py --steps 1 --warmup 1 --also-batch 0 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  for f in $(find "$OUT/p$i" -name '*counter_collection.csv'); do
    python scripts/pmc_summary.py "$f" > "$OUT/p$i.txt" && head -40 "$OUT/p$i.txt"
  done
done
