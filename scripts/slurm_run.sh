#!/bin/bash
# Multi-node launcher template (the reference's sbatch + torchrun c10d rendezvous,
# /root/reference/mingpt/slurm/slurm_run.sh), sized for 8 x MI355X per node.
#SBATCH --job-name=mingpt-mi355x
#SBATCH --nodes=2
#SBATCH --ntasks-per-node=1
#SBATCH --gpus-per-node=8
#SBATCH --cpus-per-task=64
nodes=( $( scontrol show hostnames "$SLURM_JOB_NODELIST" ) )
head_node=${nodes[0]}
head_node_ip=$(srun --nodes=1 --ntasks=1 -w "$head_node" hostname --ip-address)
export LOGLEVEL=INFO HSA_ENABLE_IPC_MODE_LEGACY=0
srun python -m torch.distributed.run --nnodes "$SLURM_NNODES" --nproc-per-node 8 \
  --max-restarts "${MAX_RESTARTS:-3}" --rdzv-id "$RANDOM" --rdzv-backend c10d --rdzv-endpoint "$head_node_ip:29500" \
  -m mingpt_distributed_amd.train --config configs/gpt2_124m.yaml \
  trainer_config.save_every_steps=500 "$@"
