set -o pipefail
mkdir -p gpurun_out/stg
for S in 0 2 4 8 12 16; do
  VARIANTS=5 LMHEAD=1 MINGPT_GEMM_STAGGER=$S timeout -k 10 120 python bench/dev/gemm_epi_variants.py >> gpurun_out/stg/w4_stagger.jsonl 2>>gpurun_out/stg/err.log || exit 1
done
cat gpurun_out/stg/w4_stagger.jsonl
