#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc2 -o a -- python3 bench/gemm_pmc_probe2.py > gpurun_out/pmc2/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM --kernel-trace --output-format csv -d gpurun_out/pmc2 -o b -- python3 bench/gemm_pmc_probe2.py > gpurun_out/pmc2/log2 2>&1 || exit $?
ls -R gpurun_out/pmc2 | head -30
