set -o pipefail
mkdir -p gpurun_out/r6b64
for r in 1 2; do
  for cfg in X=0 MINGPT_WGRAD_STREAM_TOKENS=65536; do
    env $cfg timeout -k 10 300 python bench.py --batch 64 --also-batch 0 --steps 20 --warmup 5 > gpurun_out/r6b64/${cfg}_$r.json 2> gpurun_out/r6b64/${cfg}_$r.err || { tail -5 gpurun_out/r6b64/${cfg}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/r6b64/${cfg}_$r.json $cfg $r
  done
done
