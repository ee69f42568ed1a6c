#!/bin/bash
# W4 phase stamps vs the number of tiles in flight (one round on 24 .. 255 CUs, then full size):
# does a K-tile's time grow with the CUs running (a shared limit: L2 / fabric / HBM / clock) or not
# (a per-CU one)?  Also the clock: span cycles / kernel time.   scripts/gpu/w4_occupancy_stamps.sh
set -o pipefail
cd "$(dirname "$0")/../.."
for K in 768 3072; do
  for M in 2048 8192 21760 131072; do
    timeout -k 10 60 build/bin/gemm_stamps $M 768 $K 5 0 || exit 1
  done
done
