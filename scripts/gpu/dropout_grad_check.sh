#!/bin/bash
# Model-level dropout gradient tests (tests/test_dropout_grad_gpu.py), then the same tests against
# a deliberately broken hand-off (block l's MLP-dropout seed swapped for its attention-branch seed
# in ops/fused.py, on this box's copy only): the broken run must FAIL.   dropout_grad_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-dgrad}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_dropout_grad_gpu.py -x -v --timeout 200 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
F=mingpt_distributed_amd/ops/fused.py
cp "$F" "$OUT/fused.py.orig"
sed -i 's/link_out.p, link_out.seed, link_out.dz = p_resid, seeds\[2\], None/link_out.p, link_out.seed, link_out.dz = p_resid, seeds[1], None/' "$F"
grep -q "seeds\[1\], None" "$F" || { echo "mutation not applied"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_dropout_grad_gpu.py -v --timeout 200 --timeout-method thread \
  > "$OUT/mutant.log" 2>&1
rc=$?
cp "$OUT/fused.py.orig" "$F"
grep -E "PASSED|FAILED|passed|failed" "$OUT/mutant.log" | tail -12
[ $rc -eq 1 ] || { echo "mutant run rc=$rc (expected 1: tests failed)"; exit 1; }
echo "mutant correctly detected"
