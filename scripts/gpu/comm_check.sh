set -o pipefail
mkdir -p gpurun_out/comm
timeout -k 10 400 python -u -m pytest tests/test_comm_gpu.py tests/test_dp_gpu.py -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/comm/tests.log 2>&1
s=$?; grep -E "PASS|FAIL|ERROR|passed|failed|skipped" gpurun_out/comm/tests.log | tail -30; [ $s -eq 0 ] || exit $s
for c in c10d rccl; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --also-batch 0 --comm-at-world1 --comm $c > gpurun_out/comm/bench_$c.json 2> gpurun_out/comm/bench_$c.err || { tail -20 gpurun_out/comm/bench_$c.err; exit 1; }
  tail -1 gpurun_out/comm/bench_$c.json
done
