#!/bin/bash
# One-box A/B of extension builds on the epilogue table (bench/bench_epilogue.py) and the step
# (bench.py):  TAG=x scripts/gpu/so_epi_ab.sh build/ab/A/_C.so build/ab/B/_C.so ...
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-soepi}; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
  for so in "$@"; do
    n=$(basename $(dirname $so))
    MINGPT_EXT_SO=$so timeout -k 10 300 python bench/bench_epilogue.py > "$OUT/epi_${n}_r$rep.json" 2> "$OUT/epi_${n}_r$rep.err" || { tail "$OUT/epi_${n}_r$rep.err"; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/epi_${n}_r$rep.json'))['epilogue_us_tflops']
print('$n r$rep', ' '.join('%s:%s=%.1f' % (k.split('(')[0], n2, v[0]) for k, vv in d.items() for n2, v in vv.items() if n2 in ('none','resid_p0.1','gelu_frag','dgrad_gelu_bwd_frag(NN)')))"
  done
done
for so in "$@"; do
  n=$(basename $(dirname $so))
  MINGPT_EXT_SO=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { tail "$OUT/bench_$n.err"; exit 1; }
  grep '^{' "$OUT/bench_$n.json" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$n', j['value'], j['ms_per_step'], j['extra']['batch64']['value'])"
done
