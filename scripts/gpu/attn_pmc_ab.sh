#!/bin/bash
# attention backward PMC at the bench shape (B=64) for two extension builds:
#   attn_pmc_ab.sh TAG SO_A SO_B ["COUNTERS"]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
CTR=${4:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU}
k=0
for SO in "$2" "$3"; do
  k=$((k+1))
  MINGPT_EXT_SO=$SO ATTN_B=64 timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/s$k" -o a -- python3 bench/attn_pmc.py > "$OUT/s$k.log" 2>&1 || { tail "$OUT/s$k.log"; exit 1; }
  echo "== $SO"; for f in $(find "$OUT/s$k" -name '*counter_collection.csv'); do python scripts/pmc_summary.py "$f" attn_bwd; done
done
