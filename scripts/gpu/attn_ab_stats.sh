#!/bin/bash
# Attention kernel stats at the GPT-2 bench shape for two settings of one env switch, interleaved
# in one call (rocprofv3 kernel traces of bench/dev/attn_prof.py).
#   scripts/gpu/attn_ab_stats.sh TAG VAR "VAL_A VAL_B" [rounds]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-attnab}; VAR=${2:-MINGPT_ATTN_FWD_PIPE}; VALS=${3:-"0 1"}; ROUNDS=${4:-2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${v}_$r" -o run -- \
      python3 bench/dev/attn_prof.py > "$OUT/prof_${v}_$r.log" 2>&1 || { tail -20 "$OUT/prof_${v}_$r.log"; exit 1; }
    f=$(find "$OUT/prof_${v}_$r" -name '*kernel_stats.csv' | head -1)
    echo "== $VAR=$v round $r"
    python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "attn" in r["Name"]:
        print(f'{r["Name"][:80]:80s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
  done
done
