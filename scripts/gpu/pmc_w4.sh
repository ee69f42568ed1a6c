#!/bin/bash
# W4 vs hipBLASLt counters on one NT shape (bench/gemm_pmc_w4.py), one pass per counter group
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/pmc_w4; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $OUT -o a -- python3 bench/gemm_pmc_w4.py > $OUT/log_a 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT -o b -- python3 bench/gemm_pmc_w4.py > $OUT/log_b 2>&1 || exit $?
for f in $(find $OUT -name "*counter_collection.csv"); do echo "== $f"; python scripts/pmc_summary.py $f; done > $OUT/summary.txt
cat $OUT/summary.txt
