#!/bin/bash
# Launch data-parallel training on all GPUs of one MI355X node (one process per GPU, RCCL over xGMI).
#   scripts/run_node.sh [NGPUS] [CONFIG] [overrides...]
set -euo pipefail
NGPUS=${1:-8}; CONFIG=${2:-configs/gpt2_124m.yaml}; shift $(( $# > 2 ? 2 : $# ))
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m torch.distributed.run --standalone --nnodes 1 --nproc-per-node "$NGPUS" \
  -m mingpt_distributed_amd.train --config "$CONFIG" "$@"
