set -o pipefail
mkdir -p gpurun_out/r1s2b
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r1s2b/dp.log 2>&1; s=$?; tail -5 gpurun_out/r1s2b/dp.log; [ $s -eq 0 ] || exit $s
timeout -k 10 400 python bench.py --model gpt2-xl --batch 16 --steps 5 --warmup 2 > gpurun_out/r1s2b/xl.json 2> gpurun_out/r1s2b/xl.err || { tail -20 gpurun_out/r1s2b/xl.err; exit 1; }
cat gpurun_out/r1s2b/xl.json
