#!/bin/bash
# A/B of the dQ-in-dK attention backward variants, interleaved, 3 rounds (N = 100k, 16384):
# in-tree default, diag libs given as arguments, and the separate dQ kernel (GRL_ATTN_FUSED_DQ=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
for rep in 1 2 3; do
  for v in default unfused "$@"; do
    lib=$L/libgrl.so; env=1
    [ "$v" = unfused ] && env=0
    [ "$v" != default ] && [ "$v" != unfused ] && lib=$L/diag/libgrl_$v.so
    echo "== $v" >> gpurun_out/ab_kq.log
    GRL_ATTN_FUSED_DQ=$env GRL_LIB_PATH=$lib timeout -k 10 200 python tools/probe_attn.py ${ATTN_N:-100000 16384} \
      >> gpurun_out/ab_kq.log 2>&1 || exit 1
  done
done
