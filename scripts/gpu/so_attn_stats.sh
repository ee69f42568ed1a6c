#!/bin/bash
# Attention kernel times (rocprofv3 kernel trace of bench/dev/attn_prof.py at the GPT-2 B = 128
# shape) for several extension builds on one box, interleaved over ROUNDS.
#   scripts/gpu/so_attn_stats.sh TAG ROUNDS so1 so2 ...   ("tree" = the in-tree build)
# ATTN_BWD=0 in the environment skips the backward.
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
# an entry may carry one environment setting: so@VAR=VALUE (e.g. tree@MINGPT_ATTN_FWD_DPV=0)
for r in $(seq 1 "$ROUNDS"); do
  for ent in "$@"; do
    so=${ent%%@*}; ev=""; [ "$ent" != "$so" ] && ev=${ent#*@}
    n=$(basename "$(dirname "$so")"); [ "$so" = tree ] && n=tree
    [ -n "$ev" ] && n="${n}_$(echo "$ev" | tr '=' '_')"
    if [ "$so" = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$so; fi
    env $ev timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${n}_$r" -o run -- \
      python3 bench/dev/attn_prof.py > "$OUT/${n}_$r.log" 2>&1 || { tail -20 "$OUT/${n}_$r.log"; exit 1; }
    f=$(find "$OUT/${n}_$r" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$n" "$r" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "attn" in r["Name"]:
        print(f'{sys.argv[2]:>12s} r{sys.argv[3]} {r["Name"][25:85]:60s} avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
  done
done
