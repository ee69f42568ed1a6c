set -o pipefail
mkdir -p gpurun_out/r6mini
for cfg in X=0 MINGPT_COMPUTE_PRIORITY=off MINGPT_WGRAD_STREAM=0; do
  env $cfg timeout -k 10 200 python bench.py --model gpt-mini --seq 128 --vocab 65 --batch 64 --steps 100 --warmup 20 --graph > gpurun_out/r6mini/g_$cfg.json 2> gpurun_out/r6mini/g_$cfg.err || { tail -5 gpurun_out/r6mini/g_$cfg.err; exit 1; }
  echo "graph $cfg $(tail -1 gpurun_out/r6mini/g_$cfg.json | cut -c1-160)"
  env $cfg timeout -k 10 200 python bench.py --model gpt-mini --seq 128 --vocab 65 --batch 64 --steps 100 --warmup 20 > gpurun_out/r6mini/e_$cfg.json 2> gpurun_out/r6mini/e_$cfg.err || { tail -5 gpurun_out/r6mini/e_$cfg.err; exit 1; }
  echo "eager $cfg $(tail -1 gpurun_out/r6mini/e_$cfg.json | cut -c1-160)"
done
