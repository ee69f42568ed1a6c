#!/bin/bash
# Epilogue cost table (bench/bench_epilogue.py at B = 128 tokens) and the step PMC
# (two counter passes, scripts/gpu/step_pmc.sh) on the current tree.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-epipmc}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python bench/bench_epilogue.py > "$OUT/epilogue.json" 2> "$OUT/epilogue.err" || { tail "$OUT/epilogue.err"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/epilogue.json'))['epilogue_us_tflops']
for k,v in d.items():
    print(k); [print('   %-26s %8.1f us %5d TF/s' % (n, t[0], t[1])) for n,t in v.items()]" | tee "$OUT/epilogue.txt"
bash scripts/gpu/step_pmc.sh ${TAG:-epipmc}/spmc && python scripts/step_pmc_table.py "$OUT/spmc" > "$OUT/step_pmc.txt" && head -30 "$OUT/step_pmc.txt"
