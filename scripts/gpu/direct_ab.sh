#!/bin/bash
# Round-5 experiment: W4 direct (LDS-free) epilogue builds vs the staged one (in-tree build).
#   scripts/gpu/direct_ab.sh TAG SO1 [SO2 ...]     (e.g. build/ab/direct3/_C.so)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-dab}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
SOS="tree $*"
for so in $*; do
  n=$(basename $(dirname $so))
  MINGPT_EXT_SO=$so timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_bench_scale_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests_$n.log" 2>&1
  s=$?; echo "$n tests: $(tail -1 $OUT/tests_$n.log)"
  # a crash / timeout ends the call; failed assertions are recorded and the timings still run
  if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
done
for rep in 1 2; do
  for so in $SOS; do
    n=$( [ $so = tree ] && echo tree || basename $(dirname $so) )
    if [ $so = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$so; fi
    VARIANTS=0 LMHEAD=1 timeout -k 10 300 python bench/dev/gemm_epi_variants.py > "$OUT/epi_${n}_r${rep}.jsonl" 2>&1 || { tail "$OUT/epi_${n}_r${rep}.jsonl"; exit 1; }
    echo "$n rep=$rep $(tail -1 $OUT/epi_${n}_r${rep}.jsonl)"
  done
done
for rep in 1 2; do
  for so in $SOS; do
    n=$( [ $so = tree ] && echo tree || basename $(dirname $so) )
    if [ $so = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench_${n}_r${rep}.json" 2> "$OUT/bench_${n}_r${rep}.err" || { tail "$OUT/bench_${n}_r${rep}.err"; exit 1; }
    python -c "import json; j=json.load(open('$OUT/bench_${n}_r${rep}.json')); print('$n', j['value'], j['ms_per_step'], j['extra']['batch64']['value'])"
  done
done
