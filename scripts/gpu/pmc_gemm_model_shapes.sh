#!/bin/bash
mkdir -p gpurun_out/pmc1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d gpurun_out/pmc1 -o a -- python3 bench/gemm_pmc_probe.py > gpurun_out/pmc1/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc1 -o b -- python3 bench/gemm_pmc_probe.py > gpurun_out/pmc1/log2 2>&1 || exit $?
