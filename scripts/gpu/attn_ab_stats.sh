#!/bin/bash
# Per-kernel attention times (rocprofv3, B = 128 GPT-2 shape) for several extension builds in one
# gpurun call:   scripts/gpu/attn_ab_stats.sh TAG so1 so2 ...   ("tree" = the in-tree build)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; shift
export TMPDIR=/tmp
for so in "$@"; do
  n=$(echo "$so" | tr '/' '_')
  OUT=gpurun_out/$TAG/$n
  mkdir -p "$OUT"
  if [ "$so" = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench/dev/attn_prof.py > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
  f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
  echo "== $so"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "attn" in r["Name"]:
        print(f'  {r["Name"][:70]:70s} x{r["Calls"]:>3s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
done
