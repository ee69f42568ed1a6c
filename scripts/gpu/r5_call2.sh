#!/bin/bash
# Round 5, call 2: GPU suite on the tree build, direct-epilogue A/B, decode A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5c2; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -3 "$OUT/tests.log"
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
bash scripts/gpu/direct_ab.sh r5c2 build/ab/direct3/_C.so build/ab/direct4/_C.so || exit $?
bash scripts/gpu/decode_ab.sh r5c2dec
