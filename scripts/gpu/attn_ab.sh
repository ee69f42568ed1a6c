#!/bin/bash
# attention microbench (B=32) for several extension builds, twice each, interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for so in "$@"; do
    MINGPT_EXT_SO=$so timeout -k 10 120 python bench/bench_attention.py --B 32 2>/dev/null | grep '^{' | python -c "
import json,sys
r=[json.loads(l) for l in sys.stdin]
print('$so', ' '.join(f\"p={d['p']}: fwd {d['mine_fwd_ms']} bwd {d['mine_bwd_ms']}\" for d in r))" || exit 1
  done
done
