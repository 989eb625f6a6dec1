#!/bin/bash
# A/B of the SpMM row split for F in (256, 512]: spmm_wide=1 (whole rows per wave) vs 0
# (256-column waves along grid.y) on R-MAT 1M d=512 and ER d=512 at 1M / 4M nodes.
cd $GRAFT_REPO_ROOT
for w in 1 0; do
  timeout -k 10 300 python bench.py --option spmm_wide=$w --graph rmat --nodes-per-gpu 1048576 --avg-deg 64 --dim 512 --p 0.2 --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/ab_c5s_$w.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --option spmm_wide=$w --dim 512 --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/ab_er512_$w.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --option spmm_wide=$w --dim 512 --nodes-per-gpu 4000000 --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/ab_er512_4m_$w.log 2>&1 || exit 1
done
