#!/bin/bash
# Round-3 checkpoint: attention microbench (B = 64 / 128), GPU test suite, flagship bench (B = 128
# headline + B = 64 extra), the one-rank RCCL plumbing bench, rocprofv3 kernel stats.
#   scripts/gpu/r3_check.sh TAG [--no-tests] [--no-prof]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-r3}; shift || true
TESTS=1; PROF=1
for a in "$@"; do
  case "$a" in
    --no-tests) TESTS=0 ;;
    --no-prof) PROF=0 ;;
  esac
done
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python bench/attn_ab.py > "$OUT/attn_b64.json" 2> "$OUT/attn.err" || { tail -20 "$OUT/attn.err"; exit 1; }
ATTN_B=128 timeout -k 10 200 python bench/attn_ab.py > "$OUT/attn_b128.json" 2>> "$OUT/attn.err" || { tail -20 "$OUT/attn.err"; exit 1; }
cat "$OUT"/attn_b*.json
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  s=$?; tail -3 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --also-batch 0 --comm-at-world1 > "$OUT/bench_comm1.json" 2> "$OUT/bench_comm1.err" || { tail -20 "$OUT/bench_comm1.err"; exit 1; }
cat "$OUT/bench_comm1.json"
if [ -x build/bin/xgmi_probe ]; then
  timeout -k 10 120 build/bin/xgmi_probe --max-mb 256 > "$OUT/xgmi_probe.txt" 2>&1 || { tail -20 "$OUT/xgmi_probe.txt"; exit 1; }
  python -c "import torch; print('torch.cuda.nccl.version():', torch.cuda.nccl.version())" >> "$OUT/xgmi_probe.txt" 2>/dev/null
  head -3 "$OUT/xgmi_probe.txt"
fi
if [ $PROF = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --also-batch 0 > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
  python scripts/kernel_stats.py "$OUT/prof" --steps 7 > "$OUT/kernel_stats.txt" && head -30 "$OUT/kernel_stats.txt"
fi
