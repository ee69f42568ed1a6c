#!/bin/bash
# Round 5, call 1: GPU suite on the tree build, then the direct-epilogue A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5c1; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 780 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -3 "$OUT/tests.log"
# a crash / timeout ends the call; ordinary test failures do not stop the A/B
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
bash scripts/gpu/direct_ab.sh r5c1 build/ab/direct3/_C.so build/ab/direct4/_C.so
