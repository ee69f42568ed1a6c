set -o pipefail
for so in build/ab/rd2/_C.so build/ab/stg1_e3/_C.so build/ab/stg2_e3/_C.so build/ab/stg1_e0/_C.so build/ab/rd2/_C.so; do
  echo "== $so"
  MINGPT_EXT_SO=$so timeout -k 10 120 python bench/dev/epi_scaling.py 2>/dev/null | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if d['M']>=21760: print(d['M'], d['none_us'], d['bias_us'], d['resid_us'], d['resid_drop_us'])" || exit 1
done
