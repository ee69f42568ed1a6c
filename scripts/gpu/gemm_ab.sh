#!/bin/bash
# GEMM K-sweep (bench/gemm_ksweep.py) for several extension builds, interleaved, twice each
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for so in "$@"; do
    echo "== $so"
    MINGPT_EXT_SO=$so timeout -k 10 200 python bench/gemm_ksweep.py 2>/dev/null | grep '^{' | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['N'], d['epi'], ' '.join(f\"{k}={v[0]}\" for k,v in d.items() if k.startswith('K')))" || exit 1
  done
done
