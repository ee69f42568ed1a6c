#!/bin/bash
# W4 main-loop phase stamps with the B (NOB) / A (NOA) / both fragment LDS reads removed (timing-only
# ablation builds of tools/gemm_stamps.hip, outputs wrong on purpose; the ablation switches are not in the tree)
set -o pipefail
for b in stamps_base stamps_baseDMG_ABL_NOB stamps_baseDMG_ABL_NOA stamps_baseDMG_ABL_NOADMG_ABL_NOB; do
  echo "== $b"
  timeout -k 10 60 build/bin/$b 131072 768 768 5 0 | grep -E "variant|K-tile|per tile" || exit 1
  timeout -k 10 60 build/bin/$b 131072 768 3072 5 0 | grep -E "variant|K-tile|per tile" || exit 1
done
