#!/bin/bash
# Operand-layout probe: TFLOP/s of NT vs TN (wgrad) forms, then LDS / MFMA counters of each kernel.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/pmc3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench/gemm_pmc_probe3.py > $OUT/tflops.json 2> $OUT/err.txt || exit $?
cat $OUT/tflops.json
export PMC_ITERS=2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT -o a -- python3 bench/gemm_pmc_probe3.py > $OUT/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT -o b -- python3 bench/gemm_pmc_probe3.py > $OUT/log2 2>&1 || exit $?
ls $OUT
