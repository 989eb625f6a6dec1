#!/bin/bash
# A/B of SpMM blocks per CU (bench.py --option spmm_blocks_per_cu=N) on large gathered tables:
# C5 (R-MAT 8.4M nodes, d=512, X 17 GB) and the C4 shape (ER 4M nodes, X 4 GB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for b in ${BLOCKS:-16 8 4}; do
  timeout -k 10 300 python bench.py --option spmm_blocks_per_cu=$b --graph rmat --nodes-per-gpu 8388608 --avg-deg 64 --dim 512 --p 0.2 --steps 3 \
    --warmup 1 --cpu-seconds 0 > gpurun_out/ab_occ_c5_$b.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --option spmm_blocks_per_cu=$b --nodes-per-gpu 4000000 --steps 5 --warmup 2 --cpu-seconds 0 \
    > gpurun_out/ab_occ_c4_$b.log 2>&1 || exit 1
done
