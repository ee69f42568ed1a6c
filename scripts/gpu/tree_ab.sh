#!/bin/bash
# GPU suite, bench A/B of the tree against a base tree snapshot (scripts/build_ab_tree.sh), kernel table.
#   TAG=x scripts/gpu/tree_ab.sh BASE_TREE_DIR
set -o pipefail
cd "$(dirname "$0")/../.."
BASE=$1; OUT=gpurun_out/${TAG:-treeab}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -3 "$OUT/tests.log"
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
for rep in 1 2; do
  for t in tree base; do
    B=bench.py; [ $t = base ] && B=$BASE/bench.py
    timeout -k 10 300 python $B --steps 10 --warmup 3 > "$OUT/bench_${t}_r${rep}.json" 2> "$OUT/bench_${t}_r${rep}.err" || { tail "$OUT/bench_${t}_r${rep}.err"; exit 1; }
    grep '^{' "$OUT/bench_${t}_r${rep}.json" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$t', j['value'], j['ms_per_step'], j['extra']['batch64']['value'])"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --also-batch 0 > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
python scripts/kernel_stats.py "$OUT/prof" --steps 7 > "$OUT/kernel_stats.txt" && head -24 "$OUT/kernel_stats.txt"
