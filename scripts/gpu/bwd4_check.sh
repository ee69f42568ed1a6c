#!/bin/bash
# attention tests + one-box A/B of the one-wave-per-SIMD backward (MINGPT_ATTN_BWD4=1 vs 0)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-bwd4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -15 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
for rep in 1 2; do
  for v in 1 0; do
    MINGPT_ATTN_BWD4=$v ATTN_B=128 timeout -k 10 200 python bench/attn_ab.py | sed "s/^{/{\"bwd4\": $v, /" | tee -a "$OUT/attn.jsonl" || exit 1
  done
done
for v in 1 0; do
  MINGPT_ATTN_BWD4=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof$v" -o run -- \
    python3 bench/dev/attn_prof.py > "$OUT/prof$v.log" 2>&1 || { tail -20 "$OUT/prof$v.log"; exit 1; }
  f=$(find "$OUT/prof$v" -name '*kernel_stats.csv' | head -1)
  echo "== bwd4=$v"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "attn" in r["Name"]:
        print(f'  {r["Name"][:70]:70s} x{r["Calls"]:>3s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
done
