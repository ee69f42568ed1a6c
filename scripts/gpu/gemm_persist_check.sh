#!/bin/bash
# Persistent W4 (forward layouts): GEMM GPU tests, then the step's forward GEMM shapes and the
# bench with MINGPT_GEMM_PERSIST=1 vs 0 interleaved on one box.   scripts/gpu/gemm_persist_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-gp}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread \
  > "$OUT/gemm_tests.log" 2>&1 || { tail -30 "$OUT/gemm_tests.log"; exit 1; }
tail -1 "$OUT/gemm_tests.log"
for r in 1 2; do
  for p in 1 0; do
    MINGPT_GEMM_PERSIST=$p TOKENS=131072 ROUNDS=1 timeout -k 10 300 python bench/gemm_blas_shapes.py > "$OUT/shapes_p${p}_$r.jsonl" 2> "$OUT/shapes_p${p}_$r.err" \
      || { tail -20 "$OUT/shapes_p${p}_$r.err"; exit 1; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['shape'], d['us_tflops'].get('auto'), d['us_tflops'].get('hipblaslt'))" "$OUT/shapes_p${p}_$r.jsonl" "p$p r$r"
    MINGPT_GEMM_PERSIST=$p timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench_p${p}_$r.json" 2> "$OUT/bench_p${p}_$r.err" \
      || { tail -20 "$OUT/bench_p${p}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', sys.argv[2], d['value'], d['ms_per_step'], d['extra'].get('batch64', {}).get('value'))" \
      "$OUT/bench_p${p}_$r.json" "p$p r$r"
  done
done
