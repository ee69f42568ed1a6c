#!/bin/bash
# Optimizer/forward overlap A/B on one box: GPU tests of the mode, then GPT-2 (B = 128) and
# gpt2-xl (B = 16) benches with the update in-stream (--no-opt-overlap) and overlapped, for
# the listed MINGPT_OPT_OVERLAP_BLOCKS caps, interleaved over ROUNDS.
#   scripts/gpu/opt_overlap_ab.sh TAG ROUNDS "cap1 cap2 ..."
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; ROUNDS=$2; CAPS=$3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_opt_overlap_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
run() {  # name, env, bench args
  env $2 timeout -k 10 300 python bench.py $3 > "$OUT/$1.json" 2> "$OUT/$1.err" || { tail -20 "$OUT/$1.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(f'{sys.argv[2]:>22s} {d[\"value\"]:12.1f} tok/s {d[\"ms_per_step\"]:9.3f} ms')" "$OUT/$1.json" "$1"
}
for r in $(seq 1 "$ROUNDS"); do
  run "gpt2_off_$r" "" "--steps 10 --warmup 3 --also-batch 0 --no-opt-overlap"
  run "gpt2_on_$r" "" "--steps 10 --warmup 3 --also-batch 0"
  run "xl_off_$r" "" "--model gpt2-xl --batch 16 --steps 6 --warmup 2 --also-batch 0 --no-opt-overlap"
  for c in $CAPS; do
    run "xl_on${c}_$r" "MINGPT_OPT_OVERLAP_BLOCKS=$c" "--model gpt2-xl --batch 16 --steps 6 --warmup 2 --also-batch 0"
  done
done
